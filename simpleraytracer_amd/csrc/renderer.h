// Device side of an ml_model: per-GPU scene copies, row-band split, RCCL gather.
//
// Replaces the reference's compute layer (tensorflow::Session):
// mlInfer -> Model::Infer -> Renderer::Render = H2D sample offsets per band -> prepare + trace
// kernels per GPU -> ncclGather of the bands to the first GPU -> D2H into the output Image.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "scene.h"

namespace srt {

struct CullBins;     // render.h
struct StageEvents;  // render.h

// Throws std::runtime_error("HIP error: <what>: <reason>") on failure.
void HipCheck(hipError_t err, const char* what);

// Restores the caller's current HIP device on scope exit (the C ABI must not leak a
// hipSetDevice into the host application).
class DeviceGuard {
public:
    explicit DeviceGuard(int device) {
        if (hipGetDevice(&m_prev) != hipSuccess) {
            m_prev = -1;
        }
        HipCheck(hipSetDevice(device), "hipSetDevice");
    }
    ~DeviceGuard() {
        if (m_prev >= 0) {
            (void)hipSetDevice(m_prev);
        }
    }
    DeviceGuard(const DeviceGuard&) = delete;
    DeviceGuard& operator=(const DeviceGuard&) = delete;

private:
    int m_prev = -1;
};

// GPU list from env ML_VISIBLE_DEVICES ("0,1,2"; unset = device 0; "cpu" or empty selects the CPU
// backend instead, cpu_render.h, and is never passed here). Validated against hipGetDeviceCount;
// throws when no HIP device is present.
std::vector<int> VisibleDevices();

// One device's resident copy of a scene plus its edge-record buffer.
class DeviceScene {
public:
    DeviceScene(const Scene& scene, int device);
    ~DeviceScene();
    DeviceScene(const DeviceScene&) = delete;
    DeviceScene& operator=(const DeviceScene&) = delete;

    int device() const { return m_device; }
    std::uint64_t triangles() const { return m_n; }
    const Camera& camera() const { return m_camera; }
    const float* background() const { return m_background; }

    // Edge setup for a W x H frame. The records are computed by the next Trace, on its stream
    // (fused into its first kernel); they stay valid until the next Prepare.
    void Prepare(std::size_t width, std::size_t height, hipStream_t stream);
    // Trace rows [row_begin, row_begin + row_count) of the prepared frame into RGBA, or (d_ids
    // non-null, d_rgba ignored) into hit ids for deferred shading.
    // row_interleave > 1: the band deals the frame's tile rows round-robin (render.h BandArgs).
    // id_planes >= 0: d_ids receives packed ids with that many bit planes (render.h PackedIds; the
    // cull variant; IdPlanes(triangles) must equal it).
    void Trace(const float* d_offsets, float* d_rgba, std::size_t row_begin, std::size_t row_count, int variant,
               hipStream_t stream, int* d_ids = nullptr, std::size_t row_interleave = 1, int id_planes = -1,
               bool rgba_frame_rows = false) const;
    // Deferred shading of rows [row_begin, row_begin + row_count) of the prepared frame from hit
    // ids (as Trace writes them) and sample offsets: the RGBA the fused trace would store.
    // frames > 1: a batch of that many frames of this camera, ids band-major as a gather of
    // band_rows-row bands leaves them (render.h LaunchShade), rgba [frames][row_count][width].
    // interleaved > 0: the gathered bands are that many interleaved bands. offsets_stride: floats
    // between consecutive frames' offsets (0: the batch shares d_offsets).
    void Shade(const float* d_offsets, const int* d_ids, float* d_rgba, std::size_t row_begin, std::size_t row_count,
               hipStream_t stream, std::size_t frames = 1, std::size_t band_rows = 0,
               std::size_t interleaved = 0, std::size_t offsets_stride = 0, int id_planes = -1,
               long skip_band = -1,  // skip_band: rows of that band are left as they are
               std::size_t own_bands = 0,  // and of bands [0, own_bands) (render.h LaunchShade)
               std::size_t first_rows = 0) const;  // contiguous: band 0's rows (BandSplit::first_rows)
    // `frames` (<= render.h kMaxTableFrames) frames of the prepared camera, rows [row_begin,
    // row_begin + row_count) each: frame f's offsets d_offsets[f], its RGBA d_rgba[f] or (d_ids
    // non-null) its hit ids d_ids[f]. Each frame gets the whole per-frame pipeline (record setup,
    // bins, work list, trace), as `frames` Prepare + Trace calls would; the cull variant runs all
    // frames in one launch per stage (render.h LaunchCullFrames; more than kMaxBatch frames read
    // their parameters from a device table uploaded once per call), the others frame by frame.
    void TraceBatch(const float* const* d_offsets, float* const* d_rgba, int* const* d_ids, std::size_t frames,
                    std::size_t row_begin, std::size_t row_count, int variant, hipStream_t stream,
                    std::size_t row_interleave = 1, int id_planes = -1, bool rgba_frame_rows = false,
                    const std::size_t* row_begins = nullptr) const;
    // (A frame f with d_ids non-null but d_ids[f] null and d_rgba[f] non-null is traced to RGBA;
    // rgba_frame_rows: RGBA outputs are whole frames, band rows stored at their frame rows;
    // row_begins: frame f's band starts at row_begins[f] instead -- one row count and pattern, so one
    // band shape, for every frame; cull variant, bands short of the whole frame.)

    std::size_t width() const { return m_width; }
    // The spatial order (device, triangles entries) and the time its build took at load (ms).
    const unsigned* order() const { return m_order; }
    double build_ms() const { return m_build_ms; }
    std::size_t height() const { return m_height; }

    // Stage timing: while on, Prepare and Trace bind HIP events to their kernels' dispatch
    // packets (render.h StageEvents). TakeTimes waits for them and returns the mean durations
    // (ms) of the calls timed since the previous TakeTimes, then forgets them.
    struct StageTimes {
        unsigned launches = 0;     // timed Trace calls
        double prepare_ms = 0.0;   // PrepareKernel (mean over timed Prepare calls)
        double bin_ms = 0.0;       // bin stage (cull: BinTriangles start .. WorkOrder end); 0 otherwise
        double kernel_ms = 0.0;    // the trace kernel alone
    };
    void SetTiming(bool on);
    StageTimes TakeTimes();
    // Records of the binned traces (render.h RecordMode; the env SRT_TRACE_RECORDS overrides it):
    // the frame engine sets kRecordsRecompute when it keeps one frame queue per device.
    void SetRecordMode(int mode);

private:
    int m_device;
    std::uint64_t m_n;
    Camera m_camera;
    float m_background[3];
    float* m_vertices = nullptr;
    float* m_shade = nullptr;  // shading table: 8 floats per triangle (LaunchShadeTable)
    mutable float* m_edges = nullptr;        // kEdgeFloatsPerTriangle per padded record, per frame slot
    mutable std::size_t m_edge_slots = 1;    // frame slots of m_edges (TraceBatch grows it; slot 0 = Trace's)
    unsigned* m_order = nullptr;  // record ids in spatial order (BuildSpatialOrder), for the cull bins
    unsigned* m_rank = nullptr;   // its inverse: record id -> position
    float* m_svertices = nullptr; // vertices in spatial order (svertices[i] = vertices[order[i]])
    double m_build_ms = 0.0;      // spatial order build (BuildSpatialOrder) at load
    // Per 256-position block of the spatial order: the y extent of its records' screen boxes under the
    // prepared frame (render.h LaunchBlockExtents), the band record pass's skip hint; computed on the
    // first binned trace after a Prepare (m_ext_pending). Env SRT_BLOCK_SKIP=0: never (no skip).
    mutable float2* m_block_ext = nullptr;
    mutable bool m_ext_pending = true;
    void EnsureBlockExtents(hipStream_t stream) const;
    Frame m_frame{};
    std::size_t m_width = 0;
    std::size_t m_height = 0;
    // Cull variant work buffers (render.h CullBins: tile info, bin lists, split-tile keys), grown on
    // demand by Trace; disabled by env SRT_CULL_BIN=0 (every tile then streams every record). One
    // arena per band shape in use (a band-sharing engine traces two or three shapes per batch on one
    // scene; one arena re-carved per call cost a counter fill and a new work plan every call), at most
    // kCullArenas, the least recently used re-carved for a new shape.
    // Per frame slot: frames binned in it (their parity picks the count buffer) and the trace grid
    // its work plan was built for (0: none; render.h CullBins::plan).
    struct CullSlotState {
        unsigned uses = 0;
        unsigned plan_descs = 0;
    };
    struct CullArena {
        unsigned char* work = nullptr;
        std::size_t bytes = 0;       // allocated
        std::uint64_t shape = 0;     // (width << 32) | rows of its carve-up (0: none)
        std::size_t layout = 0;      // bytes per slot (they change with the split width too)
        std::size_t zeroed = 0;      // frame slots of the carve-up whose counters are zero-filled
        std::uint64_t used = 0;      // last use (m_cull_clock)
        std::vector<CullSlotState> state;
    };
    static constexpr std::size_t kCullArenas = 4;
    mutable std::vector<CullArena> m_arenas;
    mutable std::size_t m_arena = 0;         // the arena of the current call
    mutable std::uint64_t m_cull_clock = 0;
    mutable unsigned m_cull_gen = 0;         // frames binned (render.h CullBins::gen)
    // The cull work of frame slots [0, slots) for a row_count-row band (grown, zeroed on first use
    // of a slot with this carve-up), and slot `slot`'s carve-up with a fresh frame number for a trace
    // grid of at most `descs` descriptors; it (re)builds the slot's work plan when the slot has none
    // for that grid.
    void EnsureCullWork(std::size_t slots, std::size_t row_count, hipStream_t stream) const;
    CullBins CullSlot(std::size_t slot, std::size_t row_count, unsigned descs = ~0u) const;
    void DropPlans(std::size_t slots) const;  // slots [0, slots) of every arena rebuild their plans
    void EnsureEdgeSlots(std::size_t slots, hipStream_t stream) const;
    // BVH variant: node boxes + depth bounds (render.h BvhLayout), allocated by the first bvh Trace.
    mutable unsigned char* m_bvh = nullptr;
    // Parameter tables of TraceBatch calls of more than kMaxBatch frames (render.h CullTable): a
    // ring of device tables with page-locked host staging; a staging buffer is rewritten only after
    // its previous upload has executed (its event), the device copy is protected by stream order.
    struct ParamTable {
        void* device = nullptr;
        void* host = nullptr;
        void* host_device = nullptr;  // `host` mapped into the device's address space (render.h CullTable)
        hipEvent_t uploaded = nullptr;
        std::size_t frames = 0;
        bool pending = false;
    };
    static constexpr std::size_t kParamTables = 4;
    mutable ParamTable m_tables[kParamTables];
    mutable std::size_t m_table_next = 0;
    ParamTable& AcquireTable(std::size_t frames, hipStream_t stream) const;  // after OrderAfterPrevious(stream)
    // Stage-timing events, reused: per timed Prepare (begin, end), per timed Trace (bin begin,
    // bin end, begin, end); the first m_prep_timed / m_timed entries hold pending launches.
    hipEvent_t TimingEvent(std::vector<hipEvent_t>& pool, std::size_t i) const;
    StageEvents BindStageEvents(bool prep, bool staged) const;
    bool m_timing = false;
    int m_records = 0;  // render.h RecordMode (kRecordsAuto)
    bool RecomputeRecords(std::size_t frames) const;
    // Calls on one scene are stream-ordered: the per-frame edge records and the cull work buffer
    // are shared state, so a call on another stream than the previous one first waits for it.
    void OrderAfterPrevious(hipStream_t stream) const;
    void RecordOrder(hipStream_t stream) const;
    mutable hipStream_t m_last_stream = nullptr;
    mutable bool m_used = false;
#ifndef SRT_ORDER_EVENTS
#define SRT_ORDER_EVENTS 4
#endif
    static constexpr std::size_t kOrderEvents = SRT_ORDER_EVENTS > 0 ? SRT_ORDER_EVENTS : 1;
    mutable hipEvent_t m_order_events[kOrderEvents] = {};
    mutable std::size_t m_order_next = 0;
    mutable std::vector<hipEvent_t> m_prep_events;
    mutable std::vector<hipEvent_t> m_events;
    mutable std::vector<bool> m_binned;
    mutable std::size_t m_prep_timed = 0;
    mutable bool m_prepare_pending = false;  // the full record pass has not run for the prepared frame
    mutable std::size_t m_timed = 0;
};

// Trace kernel variant from env SRT_TRACE_VARIANT ("lds" | "scalar" | "cull", default cull).
int TraceVariantFromEnv();

// How Renderer assembles a multi-device frame (env SRT_GATHER): "rccl" = the devices' hit-id bands
// gathered to the first device with ncclGather, which shades the frame and copies it out
// (default for distinct devices; on ONE device it selects a one-rank gather through the same band
// path, which puts the RCCL calls, their waits and the abort on a one-GPU box); "copy" = the same gather by device-to-device copies (default
// when a device repeats: RCCL needs distinct devices); "direct" = every device traces and shades
// its own band and copies its rows straight into the host image (no gather).
enum class GatherMode { kRccl, kCopy, kDirect };

// The device side of an ml_model (mlInfer). One device: the frame in row chunks, copies in and out
// overlapping the traces. Several (ML_VISIBLE_DEVICES): the frame's 16-row tile rows dealt
// round-robin to the devices (env SRT_BAND_ROWS=contiguous: one block each), every device traces
// its band into hit ids (4 B per pixel), the bands are gathered to the first device, which shades
// the whole frame from them (bit-identical to the fused trace) and copies it out. All launches
// from the calling thread; the RCCL gathers of all devices in one group.
class Renderer {
public:
    Renderer(const Scene& scene, std::vector<int> devices);
    ~Renderer();
    Renderer(const Renderer&) = delete;
    Renderer& operator=(const Renderer&) = delete;

    // (Re)allocate band buffers for a W x H frame. Strong guarantee: on failure the previous
    // configuration is kept.
    void Configure(std::size_t width, std::size_t height);
    bool configured() const { return m_width != 0; }

    // Render one frame: host offsets (H x W x 2) -> host RGBA (H x W x 4). Synchronous.
    // Element types from the scene's flags (kFlagInputFloat16 / kFlagOutputFloat16): float,
    // or IEEE binary16 bit patterns, converted on the device (the copies then move half the bytes).
    void Render(const void* host_offsets, void* host_rgba);
    bool input_half() const { return m_in_half; }
    bool output_half() const { return m_out_half; }

    std::size_t bands() const { return m_slots.size(); }
    GatherMode gather_mode() const { return m_gather_mode; }

private:
    struct Slot;
    struct Buffers;
    void ReleaseBuffers(Buffers& b) noexcept;
    void RenderPipelined(const void* host_offsets, void* host_rgba, std::size_t chunks);
    void RenderBands(const void* host_offsets, void* host_rgba);
    bool SyncAll() noexcept;  // bounded drain of every stream; false when one did not drain
    std::size_t BandIdBytes(std::size_t rows, std::size_t width) const;  // one band's id payload
    // Host-to-device copy of rows [0, rows) of band `i` (band-local order) from a host frame.
    void CopyBandRows(std::size_t i, const unsigned char* host, std::size_t row_bytes, unsigned char* dst,
                      hipMemcpyKind kind, bool to_host, hipStream_t stream) const;

    std::vector<std::unique_ptr<Slot>> m_slots;
    std::vector<void*> m_comms;  // ncclComm_t per slot when gathering with RCCL (nonblocking, comm.h)
    bool m_comms_aborted = false;  // a failed gather aborted them: later renders fail
    int m_id_planes = -1;          // gathered ids: packed with this many bit planes (render.h PackedIds), -1 int32
    GatherMode m_gather_mode = GatherMode::kDirect;
    bool m_interleaved = true;
    std::size_t m_band_rows = 0;  // rows of every band buffer
    int m_variant = 0;
    std::size_t m_width = 0;
    std::size_t m_height = 0;
    std::unique_ptr<Buffers> m_buf;
    bool m_in_half = false;
    bool m_out_half = false;
};

}  // namespace srt
