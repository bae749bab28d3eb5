#include "renderer.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <sstream>
#include <type_traits>

#include "comm.h"
#include "engine.h"
#include "render.h"

namespace srt {
namespace {

template <class T>
T* DeviceAlloc(std::size_t count, const char* what) {
    void* p = nullptr;
    HipCheck(hipMalloc(&p, count * sizeof(T)), what);
    return static_cast<T*>(p);
}

bool CullBinningEnabled() {
    const char* v = std::getenv("SRT_CULL_BIN");
    return v == nullptr || std::strcmp(v, "0") != 0;
}

GatherMode GatherModeFor(const std::vector<int>& devices) {
    const char* v = std::getenv("SRT_GATHER");
    if (v != nullptr && std::strcmp(v, "direct") == 0) {
        return GatherMode::kDirect;
    }
    if (v != nullptr && std::strcmp(v, "copy") == 0) {
        return GatherMode::kCopy;
    }
    if (v != nullptr && std::strcmp(v, "rccl") == 0) {
        return GatherMode::kRccl;
    }
    for (std::size_t i = 0; i < devices.size(); ++i) {
        for (std::size_t j = 0; j < i; ++j) {
            if (devices[i] == devices[j]) {
                return GatherMode::kCopy;  // one device twice: no RCCL communicator
            }
        }
    }
    return GatherMode::kRccl;
}

}  // namespace

void HipCheck(hipError_t err, const char* what) {
    if (err != hipSuccess) {
        throw std::runtime_error(std::string("HIP error: ") + what + ": " + hipGetErrorString(err));
    }
}

std::vector<int> VisibleDevices() {
    int count = 0;
    hipError_t err = hipGetDeviceCount(&count);
    if (err != hipSuccess || count <= 0) {
        throw std::runtime_error(std::string("HIP error: no HIP device available (") +
                                 (err != hipSuccess ? hipGetErrorString(err) : "device count 0") +
                                 "); set ML_VISIBLE_DEVICES=cpu to render on the CPU backend");
    }
    std::vector<int> devices;
    const char* env = std::getenv("ML_VISIBLE_DEVICES");
    if (env == nullptr || *env == '\0') {
        devices.push_back(0);
        return devices;
    }
    std::stringstream ss(env);
    std::string item;
    while (std::getline(ss, item, ',')) {
        char* end = nullptr;
        long v = std::strtol(item.c_str(), &end, 10);
        if (item.empty() || *end != '\0' || v < 0 || v >= count) {
            throw std::runtime_error("Bad ML_VISIBLE_DEVICES entry '" + item + "' (" + std::to_string(count) +
                                     " HIP devices present)");
        }
        devices.push_back(static_cast<int>(v));
    }
    if (devices.empty()) {
        devices.push_back(0);
    }
    return devices;
}

int TraceVariantFromEnv() {
    const char* v = std::getenv("SRT_TRACE_VARIANT");
    if (v != nullptr && (std::strcmp(v, "scalar") == 0 || std::strcmp(v, "1") == 0)) {
        return kTraceScalar;
    }
    if (v != nullptr && (std::strcmp(v, "lds") == 0 || std::strcmp(v, "0") == 0)) {
        return kTraceLds;
    }
    if (v != nullptr && (std::strcmp(v, "bvh") == 0 || std::strcmp(v, "3") == 0)) {
        return kTraceBvh;
    }
    return kTraceCull;
}

DeviceScene::DeviceScene(const Scene& scene, int device)
    : m_device(device), m_n(scene.triangle_count()), m_camera(scene.camera) {
    std::memcpy(m_background, scene.background, sizeof(m_background));
    DeviceGuard guard(device);
    try {
        m_vertices = DeviceAlloc<float>(m_n * 9, "hipMalloc(vertices)");
        m_shade = DeviceAlloc<float>(m_n == 0 ? 8 : m_n * 8, "hipMalloc(shading table)");
        m_edges = DeviceAlloc<float>(PaddedTriangleCount(m_n) * kEdgeFloatsPerTriangle, "hipMalloc(edges)");
        m_order = DeviceAlloc<unsigned>(m_n == 0 ? 1 : m_n, "hipMalloc(order)");
        m_rank = DeviceAlloc<unsigned>(m_n == 0 ? 1 : m_n, "hipMalloc(rank)");
        m_svertices = DeviceAlloc<float>((m_n == 0 ? 1 : m_n) * kSpatialStride, "hipMalloc(spatial vertices)");
        HipCheck(hipMemcpy(m_vertices, scene.vertices.data(), m_n * 9 * sizeof(float), hipMemcpyHostToDevice),
                 "hipMemcpy(vertices)");
        // The records' spatial order, built on the device (spatial.hip), timed.
        hipEvent_t b0 = nullptr, b1 = nullptr;
        HipCheck(hipEventCreate(&b0), "hipEventCreate(order build)");
        if (hipEventCreate(&b1) != hipSuccess) {
            (void)hipEventDestroy(b0);
            throw std::runtime_error("HIP error: hipEventCreate(order build)");
        }
        try {
            BuildSpatialOrder(m_vertices, m_n, m_camera, m_order, m_rank, m_svertices, nullptr, b0, b1);
            float ms = 0.f;
            if (m_n != 0 && hipEventElapsedTime(&ms, b0, b1) == hipSuccess) {
                m_build_ms = ms;
            }
        } catch (...) {
            (void)hipEventDestroy(b0);
            (void)hipEventDestroy(b1);
            throw;
        }
        (void)hipEventDestroy(b0);
        (void)hipEventDestroy(b1);
        if (m_n != 0) {  // the shading table from the vertices and the albedo (staged, then freed)
            float* albedo = DeviceAlloc<float>(m_n * 3, "hipMalloc(albedo)");
            hipError_t e = hipMemcpy(albedo, scene.albedo.data(), m_n * 3 * sizeof(float), hipMemcpyHostToDevice);
            if (e == hipSuccess) {
                e = LaunchShadeTable(m_vertices, albedo, m_n, m_shade, nullptr);
            }
            if (e == hipSuccess) {
                e = hipStreamSynchronize(nullptr);
            }
            (void)hipFree(albedo);
            HipCheck(e, "shading table");
        }
    } catch (...) {
        (void)hipFree(m_vertices);
        (void)hipFree(m_shade);
        (void)hipFree(m_edges);
        (void)hipFree(m_order);
        (void)hipFree(m_rank);
        (void)hipFree(m_svertices);
        throw;
    }
}

DeviceScene::~DeviceScene() {
    int prev = -1;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(m_device);
    (void)hipFree(m_vertices);
    (void)hipFree(m_shade);
    (void)hipFree(m_edges);
    (void)hipFree(m_order);
    (void)hipFree(m_rank);
    (void)hipFree(m_svertices);
    (void)hipFree(m_block_ext);
    for (CullArena& a : m_arenas) {
        (void)hipFree(a.work);
    }
    (void)hipFree(m_bvh);
    for (hipEvent_t e : m_events) {
        (void)hipEventDestroy(e);
    }
    for (hipEvent_t e : m_prep_events) {
        (void)hipEventDestroy(e);
    }
    for (hipEvent_t e : m_order_events) {
        if (e != nullptr) {
            (void)hipEventDestroy(e);
        }
    }
    for (ParamTable& t : m_tables) {
        if (t.uploaded != nullptr) {
            (void)hipEventSynchronize(t.uploaded);
            (void)hipEventDestroy(t.uploaded);
        }
        (void)hipFree(t.device);
        (void)hipHostFree(t.host);
    }
    if (prev >= 0) {
        (void)hipSetDevice(prev);
    }
}

void DeviceScene::Prepare(std::size_t width, std::size_t height, hipStream_t stream) {
    if (width == 0 || height == 0) {
        throw std::runtime_error("Prepare: frame dimensions must be non-zero");
    }
    if (width != m_width || height != m_height) {
        DropPlans(~std::size_t{0});  // (a plan is scheduling only; a new shape deserves a new one)
    }
    m_frame = MakeFrame(m_camera, width, height);
    m_width = width;
    m_height = height;
    // Deferred: the next Trace enqueues the record setup on its stream (the binned cull path
    // computes the records inside its bin kernel on every call, render.hip PrepareBinKernel).
    (void)stream;
    m_prepare_pending = true;
    m_ext_pending = true;
}

// The block extents of the prepared frame, once per Prepare (on the first binned trace's stream,
// before its launches). They depend on the scene, its camera and W x H only, like the spatial order.
void DeviceScene::EnsureBlockExtents(hipStream_t stream) const {
    static const bool enabled = [] {
        const char* v = std::getenv("SRT_BLOCK_SKIP");
        return v == nullptr || std::strcmp(v, "0") != 0;
    }();
    if (!enabled || !m_ext_pending || m_n == 0) {
        return;
    }
    if (m_block_ext == nullptr) {
        m_block_ext = DeviceAlloc<float2>(BlockExtentCount(m_n), "hipMalloc(block extents)");
    }
    HipCheck(LaunchBlockExtents(m_svertices, m_n, m_frame, m_block_ext, stream), "block extents launch");
    m_ext_pending = false;
}

void DeviceScene::OrderAfterPrevious(hipStream_t stream) const {
    if (m_used && stream != m_last_stream) {
#if SRT_ORDER_EVENTS == 0
        HipCheck(hipEventRecord(m_order_events[0], m_last_stream), "hipEventRecord(scene order)");
#endif
        HipCheck(hipStreamWaitEvent(stream, m_order_events[m_order_next], 0), "hipStreamWaitEvent(scene order)");
    }
#if SRT_ORDER_EVENTS == 0
    if (m_order_events[0] == nullptr) {
        HipCheck(hipEventCreateWithFlags(&m_order_events[0], hipEventDisableTiming), "hipEventCreate(scene order)");
    }
    m_used = true;
    m_last_stream = stream;
#endif
}

// Marks the end of this call's work on `stream`: the next call on another stream waits for it. The
// event is recorded on the call's own stream, so the library never touches a stream after the call
// that was given it has returned (the caller may destroy it). A ring of events: recording an
// event whose previous record is still pending can stall the host, so consecutive calls use
// different events and only the newest is waited on.
void DeviceScene::RecordOrder(hipStream_t stream) const {
#if SRT_ORDER_EVENTS > 0
    const std::size_t k = (m_order_next + 1) % kOrderEvents;
    if (m_order_events[k] == nullptr) {
        HipCheck(hipEventCreateWithFlags(&m_order_events[k], hipEventDisableTiming), "hipEventCreate(scene order)");
    }
    HipCheck(hipEventRecord(m_order_events[k], stream), "hipEventRecord(scene order)");
    m_order_next = k;
    m_used = true;
    m_last_stream = stream;
#else
    (void)stream;
#endif
}

void DeviceScene::Shade(const float* d_offsets, const int* d_ids, float* d_rgba, std::size_t row_begin,
                        std::size_t row_count, hipStream_t stream, std::size_t frames, std::size_t band_rows,
                        std::size_t interleaved, std::size_t offsets_stride, int id_planes, long skip_band,
                        std::size_t own_bands, std::size_t first_rows) const {
    if (id_planes >= 0 && id_planes != IdPlanes(m_n)) {
        throw std::runtime_error("Shade: packed ids of this scene have " + std::to_string(IdPlanes(m_n)) + " bit planes");
    }
    if (m_width == 0) {
        throw std::runtime_error("Shade: Prepare() has not been called");
    }
    if (interleaved > 0) {  // every band the ids hold (from own_bands on) fits a band_rows-row buffer
        bool fits = row_begin == 0;
        for (std::size_t j = own_bands; j < interleaved && fits; ++j) {
            fits = band_rows >= InterleavedBandRows(m_height, interleaved, j);
        }
        if (!fits) {
            throw std::runtime_error("Shade: interleaved bands cover the whole frame in band_rows-row buffers");
        }
    }
    if (row_begin + row_count > m_height) {
        throw std::runtime_error("Shade: row band outside the frame");
    }
    if (band_rows > row_count || frames > 65535) {
        throw std::runtime_error("Shade: band_rows exceeds the rows shaded, or more than 65535 frames");
    }
    if (first_rows > row_count || (first_rows != 0 && interleaved > 0)) {
        throw std::runtime_error("Shade: first_rows exceeds the rows shaded, or with interleaved bands");
    }
    if (row_count == 0 || frames == 0) {
        return;
    }
    OrderAfterPrevious(stream);
    BandArgs band{d_offsets, d_rgba, m_width, m_height, row_begin, row_count, const_cast<int*>(d_ids)};
    band.id_planes = id_planes;
    HipCheck(LaunchShade(m_vertices, m_shade, m_edges, m_n, m_frame, m_background, band, stream, frames, band_rows,
                         interleaved, offsets_stride, skip_band, own_bands, first_rows),
             "shade kernel launch");
    RecordOrder(stream);
}

// Grow-only cull work for `slots` frame slots of one carve-up (render.h CullBins; counters reset
// themselves, so a slot's counters are zero-filled only on its first use with this carve-up), in the
// arena of this band shape.
void DeviceScene::EnsureCullWork(std::size_t slots, std::size_t row_count, hipStream_t stream) const {
    const std::size_t bytes = CullBinBytes(m_n, m_width, row_count);
    const std::uint64_t shape = (static_cast<std::uint64_t>(m_width) << 32) | row_count;
    std::size_t pick = m_arenas.size();
    for (std::size_t i = 0; i < m_arenas.size(); ++i) {
        if (m_arenas[i].shape == shape && m_arenas[i].layout == bytes) {
            pick = i;
        }
    }
    if (pick == m_arenas.size()) {  // a new shape: a new arena, or the least recently used one re-carved
        if (m_arenas.size() < kCullArenas) {
            m_arenas.emplace_back();
        } else {
            pick = 0;
            for (std::size_t i = 1; i < m_arenas.size(); ++i) {
                pick = m_arenas[i].used < m_arenas[pick].used ? i : pick;
            }
        }
        CullArena& a = m_arenas[pick];
        a.shape = shape;
        a.layout = bytes;
        a.zeroed = 0;  // (stream order: earlier launches on this arena ran before its counters are reset)
    }
    CullArena& a = m_arenas[pick];
    if (slots * bytes > a.bytes) {
        HipCheck(hipStreamSynchronize(stream), "hipStreamSynchronize(cull work)");
        (void)hipFree(a.work);
        a.work = nullptr;
        a.bytes = 0;
        a.work = DeviceAlloc<unsigned char>(slots * bytes, "hipMalloc(cull work)");
        a.bytes = slots * bytes;
        a.zeroed = 0;
    }
    if (slots > a.zeroed) {
        // Only each slot's leading counters (render.h CullBins): zeroing whole slots (~30 MB each,
        // mostly split-key slices) cost 0.4-0.5 ms per 64-frame batch whenever a shape was re-carved.
        HipCheck(hipMemset2DAsync(a.work + a.zeroed * bytes, bytes, 0, CullBinCounterBytes(m_n, m_width, row_count),
                                  slots - a.zeroed, stream),
                 "hipMemset2DAsync(cull work)");
        a.state.resize(std::max(a.state.size(), slots));
        for (std::size_t k = a.zeroed; k < slots; ++k) {
            a.state[k] = CullSlotState{};  // zeroed: no plan
        }
        a.zeroed = slots;
    }
    a.used = ++m_cull_clock;
    m_arena = pick;
}

void DeviceScene::DropPlans(std::size_t slots) const {
    for (CullArena& a : m_arenas) {
        for (std::size_t k = 0; k < slots && k < a.state.size(); ++k) {
            a.state[k].plan_descs = 0;
        }
    }
}


CullBins DeviceScene::CullSlot(std::size_t slot, std::size_t row_count, unsigned descs) const {
    CullArena& a = m_arenas.at(m_arena);  // (EnsureCullWork picked and sized it)
    CullSlotState& st = a.state.at(slot);
    CullBins bins = CullBinLayout(a.work + slot * a.layout, m_n, m_width, row_count, st.uses & 1u);
    bins.descs = std::min(bins.descs, descs);
    bins.plan = st.plan_descs != bins.descs;  // (render.hip WorkPlan: the launch may order anyway)
    st.plan_descs = bins.descs;
    ++st.uses;
    bins.order = m_order;
    bins.svertices = m_svertices;
    bins.block_ext = m_ext_pending ? nullptr : m_block_ext;
    m_cull_gen = m_cull_gen + 1u == 0u ? 1u : m_cull_gen + 1u;
    bins.gen = m_cull_gen;
    return bins;
}

// Edge records for `slots` frame slots (slot 0 is the one Prepare / Trace / Shade use). Growing
// drops the prepared records, so the next trace recomputes them.
void DeviceScene::EnsureEdgeSlots(std::size_t slots, hipStream_t stream) const {
    if (slots <= m_edge_slots) {
        return;
    }
    HipCheck(hipStreamSynchronize(stream), "hipStreamSynchronize(edges)");
    const std::size_t floats = PaddedTriangleCount(m_n) * kEdgeFloatsPerTriangle;
    float* grown = DeviceAlloc<float>(slots * floats, "hipMalloc(edges)");
    (void)hipFree(m_edges);
    m_edges = grown;
    m_edge_slots = slots;
    m_prepare_pending = true;
}

DeviceScene::ParamTable& DeviceScene::AcquireTable(std::size_t frames, hipStream_t stream) const {
    ParamTable& t = m_tables[m_table_next];
    m_table_next = (m_table_next + 1) % kParamTables;
    if (t.pending) {
        HipCheck(hipEventSynchronize(t.uploaded), "hipEventSynchronize(parameter table)");
        t.pending = false;
    }
    if (t.frames < frames) {
        // Every table of the ring grows at once (one stall, on the first large call, instead of one at
        // the first use of each). Launches queued earlier may still read an old device table. They all
        // run before `stream`'s current end (calls on one scene are stream-ordered: OrderAfterPrevious
        // ran first), so draining this stream suffices -- never a device-wide sync from an engine worker
        // (other workers' queues and RCCL kernels waiting on peers would be waited for too).
        HipCheck(hipStreamSynchronize(stream), "hipStreamSynchronize(parameter table)");
        const std::size_t bytes = CullTableBytes(frames);
        for (ParamTable& r : m_tables) {
            if (r.frames >= frames) {
                continue;
            }
            r.pending = false;  // (its uploads ran: the stream is drained)
            (void)hipFree(r.device);
            (void)hipHostFree(r.host);
            r.device = nullptr;
            r.host = nullptr;
            r.host_device = nullptr;
            r.frames = 0;
            HipCheck(hipMalloc(&r.device, bytes), "hipMalloc(parameter table)");
            // Mapped and fine-grained (coherent): the upload kernel reads it over the bus, uncached,
            // so a table rewritten for a later launch is never read stale from the L2.
            HipCheck(hipHostMalloc(&r.host, bytes, hipHostMallocMapped | hipHostMallocCoherent),
                     "hipHostMalloc(parameter table)");
            HipCheck(hipHostGetDevicePointer(&r.host_device, r.host, 0), "hipHostGetDevicePointer(parameter table)");
            r.frames = frames;
        }
    }
    if (t.uploaded == nullptr) {
        HipCheck(hipEventCreateWithFlags(&t.uploaded, hipEventDisableTiming), "hipEventCreate(parameter table)");
    }
    return t;
}

void DeviceScene::TraceBatch(const float* const* d_offsets, float* const* d_rgba, int* const* d_ids, std::size_t frames,
                             std::size_t row_begin, std::size_t row_count, int variant, hipStream_t stream,
                             std::size_t row_interleave, int id_planes, bool rgba_frame_rows,
                             const std::size_t* row_begins) const {
    if (id_planes >= 0 && (id_planes != IdPlanes(m_n) || variant != kTraceCull)) {
        throw std::runtime_error("TraceBatch: packed ids need the cull variant and " + std::to_string(IdPlanes(m_n)) +
                                 " bit planes for this scene");
    }
    if (m_width == 0) {
        throw std::runtime_error("TraceBatch: Prepare() has not been called");
    }
    if (!BandFits(row_begin, row_count, row_interleave, m_height)) {
        throw std::runtime_error("TraceBatch: row band outside the frame");
    }
    bool same_begin = true;  // render.hip LaunchCullFrames: per-frame first rows compute their tile info first
    for (std::size_t f = 0; row_begins != nullptr && f < frames; ++f) {
        if (!BandFits(row_begins[f], row_count, row_interleave, m_height)) {
            throw std::runtime_error("TraceBatch: per-frame bands must lie inside the frame");
        }
        same_begin = same_begin && row_begins[f] == row_begins[0];
    }
    if (row_begins != nullptr && (variant != kTraceCull || !CullBinningEnabled() || !CullBinnable(m_width, row_count))) {
        throw std::runtime_error("TraceBatch: per-frame bands need the binned cull variant");
    }
    if (frames > static_cast<std::size_t>(kMaxTableFrames)) {
        throw std::runtime_error("TraceBatch: at most " + std::to_string(kMaxTableFrames) + " frames per batch");
    }
    if (frames == 0 || row_count == 0) {
        return;
    }
    if (variant != kTraceCull || !CullBinningEnabled() || !CullBinnable(m_width, row_count)) {
        for (std::size_t f = 0; f < frames; ++f) {  // frame by frame, each with its own record setup
            m_prepare_pending = true;
            int* ids_f = d_ids != nullptr ? d_ids[f] : nullptr;
            Trace(d_offsets[f], d_rgba != nullptr ? d_rgba[f] : nullptr, row_begin, row_count, variant, stream, ids_f,
                  row_interleave, ids_f != nullptr ? id_planes : -1, rgba_frame_rows);
        }
        return;
    }
    OrderAfterPrevious(stream);
    EnsureEdgeSlots(frames, stream);
    EnsureCullWork(frames, row_count, stream);
    EnsureBlockExtents(stream);
    std::vector<CullBins> bins(frames);
    std::vector<CullFrame> cf(frames);
    const std::size_t floats = PaddedTriangleCount(m_n) * kEdgeFloatsPerTriangle;
    // The trace grid for the whole batch: its frames' parts together fill the chip sooner (a
    // 135-row band alone splits 5 ways; eight of them do not need to).
    const unsigned batch_descs = CullDescriptors(CullTiles(m_width, row_count), frames);
    const bool recompute = RecomputeRecords(frames);
    for (std::size_t f = 0; f < frames; ++f) {
        bins[f] = CullSlot(f, row_count, batch_descs);
        bins[f].recompute = recompute;
        cf[f].edges = m_edges + f * floats;
        cf[f].bins = &bins[f];
        cf[f].band = BandArgs{d_offsets[f], d_rgba != nullptr ? d_rgba[f] : nullptr, m_width, m_height,
                              row_begins != nullptr ? row_begins[f] : row_begin, row_count,
                              d_ids != nullptr ? d_ids[f] : nullptr, row_interleave, id_planes, rgba_frame_rows};
    }
    const StageEvents ev = BindStageEvents(
        !same_begin || !CullFusedInfo(row_begins != nullptr ? row_begins[0] : row_begin, row_count, m_height, row_interleave),
        true);
    ParamTable* table = frames > static_cast<std::size_t>(kMaxBatch) ? &AcquireTable(frames, stream) : nullptr;
    const CullTable ct{table != nullptr ? table->device : nullptr, table != nullptr ? table->host : nullptr,
                       table != nullptr ? table->frames : 0, table != nullptr ? table->host_device : nullptr,
                       table != nullptr ? table->uploaded : nullptr};
    const hipError_t launched = LaunchCullFrames(cf.data(), frames, m_n, m_vertices, m_shade, m_frame, m_background,
                                                 m_rank, stream, m_timing ? &ev : nullptr,
                                                 table != nullptr ? &ct : nullptr);
    if (launched != hipSuccess) {
        DropPlans(frames);
    }
    HipCheck(launched, "batched trace launch");
    if (table != nullptr) {
        table->pending = true;  // (LaunchCullFrames recorded `uploaded` after the upload)
    }
    RecordOrder(stream);
}

void DeviceScene::Trace(const float* d_offsets, float* d_rgba, std::size_t row_begin, std::size_t row_count,
                        int variant, hipStream_t stream, int* d_ids, std::size_t row_interleave, int id_planes,
                        bool rgba_frame_rows) const {
    if (id_planes >= 0 && (d_ids == nullptr || id_planes != IdPlanes(m_n) || variant != kTraceCull)) {
        throw std::runtime_error("Trace: packed ids need an id output, the cull variant and " +
                                 std::to_string(IdPlanes(m_n)) + " bit planes for this scene");
    }
    if (m_width == 0) {
        throw std::runtime_error("Trace: Prepare() has not been called");
    }
    if (!BandFits(row_begin, row_count, row_interleave, m_height)) {
        throw std::runtime_error("Trace: row band outside the frame");
    }
    OrderAfterPrevious(stream);
    BandArgs band{d_offsets, d_rgba, m_width, m_height, row_begin, row_count, d_ids, row_interleave, id_planes,
                  rgba_frame_rows};
    CullBins bins{};
    const CullBins* use_bins = nullptr;
    if (variant == kTraceCull && row_count != 0 && CullBinningEnabled() && CullBinnable(m_width, row_count)) {
        EnsureCullWork(1, row_count, stream);
        EnsureBlockExtents(stream);
        bins = CullSlot(0, row_count);
        bins.recompute = RecomputeRecords(1);
        use_bins = &bins;
    }
    if (variant == kTraceBvh && m_bvh == nullptr && row_count != 0) {
        m_bvh = DeviceAlloc<unsigned char>(BvhBytes(m_n), "hipMalloc(bvh)");
    }
    // The full record pass for every path but the binned cull one, which computes its records in
    // its bin kernel (its "prepare" stage is the tile-info kernel).
    const bool prepare = use_bins == nullptr && m_prepare_pending && row_count != 0;
    const bool fused_info = use_bins != nullptr && CullFusedInfo(row_begin, row_count, m_height, row_interleave);
    const StageEvents ev = BindStageEvents(prepare || (use_bins != nullptr && row_count != 0 && !fused_info),
                                           use_bins != nullptr || (variant == kTraceBvh && m_n != 0));
    const hipError_t launched = LaunchTrace(m_edges, m_n, m_vertices, m_shade, m_frame, m_background, band, variant,
                                            use_bins, stream, m_timing ? &ev : nullptr, prepare ? m_rank : nullptr,
                                            m_bvh);
    if (launched != hipSuccess && use_bins != nullptr) {
        DropPlans(1);
    }
    HipCheck(launched, "trace kernel launch");
    if (prepare) {
        m_prepare_pending = false;
    }
    RecordOrder(stream);
}

// With stage timing on: events for one traced call (a batch counts as one call).
StageEvents DeviceScene::BindStageEvents(bool prep, bool staged) const {
    StageEvents ev{};
    if (!m_timing) {
        return ev;
    }
    if (prep) {
        ev.prep_begin = TimingEvent(m_prep_events, 2 * m_prep_timed);
        ev.prep_end = TimingEvent(m_prep_events, 2 * m_prep_timed + 1);
        ++m_prep_timed;
    }
    const std::size_t k = 4 * m_timed;
    ev.bin_begin = staged ? TimingEvent(m_events, k) : nullptr;
    ev.bin_end = staged ? TimingEvent(m_events, k + 1) : nullptr;
    ev.begin = TimingEvent(m_events, k + 2);
    ev.end = TimingEvent(m_events, k + 3);
    if (m_binned.size() <= m_timed) {
        m_binned.resize(m_timed + 1);
    }
    m_binned[m_timed] = staged;
    ++m_timed;
    return ev;
}

hipEvent_t DeviceScene::TimingEvent(std::vector<hipEvent_t>& pool, std::size_t i) const {
    while (pool.size() <= i) {
        hipEvent_t e = nullptr;
        HipCheck(hipEventCreate(&e), "hipEventCreate(stage timing)");
        pool.push_back(e);
    }
    return pool[i];
}

void DeviceScene::SetTiming(bool on) {
    m_timing = on;
}

namespace {
// SRT_TRACE_RECORDS: stored | recompute | auto (render.h RecordMode); -1 when unset. Read per launch
// (like SRT_CULL_BIN), so a process can compare the modes.
int RecordModeFromEnv() {
    const char* e = std::getenv("SRT_TRACE_RECORDS");
    if (e == nullptr || *e == '\0') {
        return -1;
    }
    const std::string v(e);
    if (v == "auto") {
        return static_cast<int>(kRecordsAuto);
    }
    if (v == "stored") {
        return static_cast<int>(kRecordsStored);
    }
    if (v == "recompute") {
        return static_cast<int>(kRecordsRecompute);
    }
    throw std::runtime_error("SRT_TRACE_RECORDS must be stored, recompute or auto, got '" + v + "'");
}
}  // namespace

void DeviceScene::SetRecordMode(int mode) {
    if (mode != kRecordsAuto && mode != kRecordsStored && mode != kRecordsRecompute) {
        throw std::runtime_error("SetRecordMode: unknown record mode " + std::to_string(mode));
    }
    m_records = mode;
}

// Whether a binned launch of `frames` frames has its trace recompute the records: the bin launch
// then writes 16 B per record instead of 64, which shortens it by a fifth, and the trace rebuilds each
// candidate's record (~5 % longer). It pays where the bin launch is on the critical path: a launch of one
// frame, or an engine with one frame queue (nothing overlaps its bin launches).
bool DeviceScene::RecomputeRecords(std::size_t frames) const {
    const int env = RecordModeFromEnv();
    const int mode = env >= 0 ? env : m_records;
    return mode == kRecordsRecompute || (mode == kRecordsAuto && frames == 1);
}

DeviceScene::StageTimes DeviceScene::TakeTimes() {
    auto elapsed = [](hipEvent_t a, hipEvent_t b) {
        HipCheck(hipEventSynchronize(b), "hipEventSynchronize(stage timing)");
        float ms = 0.f;
        HipCheck(hipEventElapsedTime(&ms, a, b), "hipEventElapsedTime(stage timing)");
        return static_cast<double>(ms);
    };
    StageTimes t;
    for (std::size_t i = 0; i < m_prep_timed; ++i) {
        t.prepare_ms += elapsed(m_prep_events[2 * i], m_prep_events[2 * i + 1]);
    }
    std::size_t binned = 0;
    for (std::size_t i = 0; i < m_timed; ++i) {
        if (m_binned[i]) {
            t.bin_ms += elapsed(m_events[4 * i], m_events[4 * i + 1]);
            ++binned;
        }
        t.kernel_ms += elapsed(m_events[4 * i + 2], m_events[4 * i + 3]);
    }
    t.launches = static_cast<unsigned>(m_timed);
    t.prepare_ms /= m_prep_timed != 0 ? static_cast<double>(m_prep_timed) : 1.0;
    t.bin_ms /= binned != 0 ? static_cast<double>(binned) : 1.0;
    t.kernel_ms /= m_timed != 0 ? static_cast<double>(m_timed) : 1.0;
    m_prep_timed = 0;
    m_timed = 0;
    return t;
}

struct Renderer::Slot {
    int device = 0;
    hipStream_t stream = nullptr;
    std::unique_ptr<DeviceScene> scene;
    std::size_t band = 0;  // band index (= slot index)
    std::size_t row_begin = 0;
    std::size_t row_count = 0;
    // Pipelined single-device render (Renderer::RenderPipelined): copy streams and per-chunk
    // events (H2D done, chunk traced); `traced[0]` also orders the device-copy gather.
    hipStream_t copy_in = nullptr;
    hipStream_t copy_out = nullptr;
    std::vector<hipEvent_t> in_done;
    std::vector<hipEvent_t> traced;
    hipEvent_t done = nullptr;  // band path: end of the frame's work on this device (polled, comm.h)
};

// The buffers of one frame size (Configure builds a new set before releasing the old one).
struct Renderer::Buffers {
    std::vector<int> devices;
    std::vector<float*> offsets;           // band rows x W x 2 per slot (one device: the frame)
    std::vector<std::uint16_t*> offsets16;  // FLOAT16 input: H2D staging
    std::vector<float*> rgba;              // band rows x W x 4 (direct mode, one device)
    std::vector<std::uint16_t*> rgba16;    // FLOAT16 output staging of rgba
    std::vector<int*> ids;                 // band rows x W hit ids (gather modes)
    int root = 0;
    float* full = nullptr;                 // root: the frame's offsets (shading), H x W x 2
    std::uint16_t* full16 = nullptr;
    int* gather = nullptr;                 // root: bands x band rows x W gathered ids
    float* frame = nullptr;                // root: H x W x 4 shaded frame
    std::uint16_t* frame16 = nullptr;
};

namespace {
// Row chunks of the pipelined single-device render: env SRT_E2E_CHUNKS (1 = no pipelining).
std::size_t E2eChunks() {
    const char* v = std::getenv("SRT_E2E_CHUNKS");
    const long c = v == nullptr || *v == '\0' ? 4 : std::strtol(v, nullptr, 10);
    return c < 1 ? 1 : (c > 16 ? 16 : static_cast<std::size_t>(c));
}

bool InterleavedFromEnv() {
    const char* v = std::getenv("SRT_BAND_ROWS");
    return v == nullptr || std::strcmp(v, "contiguous") != 0;
}

template <class T>
void FreeOn(int device, T*& p) noexcept {
    if (p != nullptr) {
        (void)hipSetDevice(device);
        (void)hipFree(p);
        p = nullptr;
    }
}
}  // namespace

Renderer::Renderer(const Scene& scene, std::vector<int> devices)
    : m_interleaved(InterleavedFromEnv()),
      m_variant(TraceVariantFromEnv()),
      m_in_half((scene.flags & kFlagInputFloat16) != 0u),
      m_out_half((scene.flags & kFlagOutputFloat16) != 0u) {
    for (std::size_t i = 0; i < devices.size(); ++i) {
        auto slot = std::make_unique<Slot>();
        slot->device = devices[i];
        slot->band = i;
        DeviceGuard guard(devices[i]);
        HipCheck(hipStreamCreateWithFlags(&slot->stream, hipStreamNonBlocking), "hipStreamCreate");
        m_slots.push_back(std::move(slot));
        m_slots.back()->scene = std::make_unique<DeviceScene>(scene, devices[i]);
    }
    m_gather_mode = m_slots.size() > 1 ? GatherModeFor(devices) : GatherMode::kDirect;
    if (m_slots.size() == 1) {  // SRT_GATHER=rccl on one device: the band path with a one-rank gather (tests)
        const char* v = std::getenv("SRT_GATHER");
        if (v != nullptr && std::strcmp(v, "rccl") == 0) {
            m_gather_mode = GatherMode::kRccl;
        }
    }
    // Gathered payload: packed ids (render.h PackedIds: 16 + k bits per pixel) with the cull variant
    // (env SRT_EXCHANGE_IDS=32: int32 ids), about half the bytes over xGMI.
    {
        const char* v = std::getenv("SRT_EXCHANGE_IDS");
        const bool force32 = v != nullptr && std::strcmp(v, "32") == 0;
        m_id_planes = m_variant == kTraceCull && !force32 ? IdPlanes(scene.triangle_count()) : -1;
    }
    if (m_gather_mode == GatherMode::kRccl) {
        try {
            m_comms = CommInitAll(devices);  // nonblocking communicators (comm.h)
        } catch (const std::exception& e) {
            throw std::runtime_error(std::string(e.what()) + " (a repeated device needs SRT_GATHER=copy or direct)");
        }
    }
}

Renderer::~Renderer() {
    if (!SyncAll()) {
        // Work that never finished still uses the device buffers (hipFree would wait for it): leak them.
        CommAbortAll(m_comms);
        for (auto& slot : m_slots) {
            (void)slot->scene.release();
        }
        (void)m_buf.release();
        return;
    }
    if (m_buf) {
        ReleaseBuffers(*m_buf);
    }
    CommDestroyAll(m_comms);
    for (auto& slot : m_slots) {
        (void)hipSetDevice(slot->device);
        slot->scene.reset();
        if (slot->done != nullptr) {
            (void)hipEventDestroy(slot->done);
        }
        for (hipEvent_t e : slot->in_done) {
            (void)hipEventDestroy(e);
        }
        for (hipEvent_t e : slot->traced) {
            (void)hipEventDestroy(e);
        }
        if (slot->copy_in != nullptr) {
            (void)hipStreamDestroy(slot->copy_in);
        }
        if (slot->copy_out != nullptr) {
            (void)hipStreamDestroy(slot->copy_out);
        }
        (void)hipStreamDestroy(slot->stream);
    }
}

std::size_t Renderer::BandIdBytes(std::size_t rows, std::size_t width) const {
    // int32 ids, or one packed band frame (a multiple of 256 B) -- in whole ints either way
    const std::size_t b = m_id_planes >= 0 ? PackedIdLayout(m_id_planes, rows, width).bytes : rows * width * sizeof(int);
    return (b + sizeof(int) - 1) / sizeof(int) * sizeof(int);
}

void Renderer::ReleaseBuffers(Buffers& b) noexcept {
    for (std::size_t i = 0; i < b.devices.size(); ++i) {
        FreeOn(b.devices[i], b.offsets[i]);
        FreeOn(b.devices[i], b.offsets16[i]);
        FreeOn(b.devices[i], b.rgba[i]);
        FreeOn(b.devices[i], b.rgba16[i]);
        FreeOn(b.devices[i], b.ids[i]);
    }
    FreeOn(b.root, b.full);
    FreeOn(b.root, b.full16);
    FreeOn(b.root, b.gather);
    FreeOn(b.root, b.frame);
    FreeOn(b.root, b.frame16);
}

void Renderer::Configure(std::size_t width, std::size_t height) {
    const std::size_t bands = m_slots.size();
    const bool multi = bands > 1;
    const bool gather = (multi || m_gather_mode == GatherMode::kRccl) && m_gather_mode != GatherMode::kDirect;
    const BandSplit split = BandSplit::Make(height, bands, m_interleaved);
    const std::size_t band_rows = split.BufferRows();
    // Allocate everything new before releasing the old buffers (strong guarantee).
    auto nb = std::make_unique<Buffers>();
    nb->offsets.assign(bands, nullptr);
    nb->offsets16.assign(bands, nullptr);
    nb->rgba.assign(bands, nullptr);
    nb->rgba16.assign(bands, nullptr);
    nb->ids.assign(bands, nullptr);
    nb->root = m_slots.front()->device;
    for (auto& sp : m_slots) {
        nb->devices.push_back(sp->device);
    }
    auto alloc = [](auto*& p, std::size_t count, const char* what) {
        void* q = nullptr;
        HipCheck(hipMalloc(&q, (count == 0 ? 1 : count) * sizeof(*p)), what);
        p = static_cast<std::remove_reference_t<decltype(p)>>(q);
    };
    try {
        for (std::size_t i = 0; i < bands; ++i) {
            DeviceGuard guard(m_slots[i]->device);
            alloc(nb->offsets[i], band_rows * width * 2, "hipMalloc(band offsets)");
            if (m_in_half) {
                alloc(nb->offsets16[i], band_rows * width * 2, "hipMalloc(band offsets f16)");
            }
            if (gather) {
                alloc(nb->ids[i], BandIdBytes(band_rows, width) / sizeof(int), "hipMalloc(band ids)");
            } else {
                alloc(nb->rgba[i], band_rows * width * 4, "hipMalloc(band framebuffer)");
                if (m_out_half) {
                    alloc(nb->rgba16[i], band_rows * width * 4, "hipMalloc(band framebuffer f16)");
                }
            }
        }
        if (gather) {
            DeviceGuard guard(nb->root);
            alloc(nb->full, height * width * 2, "hipMalloc(frame offsets)");
            if (m_in_half) {
                alloc(nb->full16, height * width * 2, "hipMalloc(frame offsets f16)");
            }
            alloc(nb->gather, bands * BandIdBytes(band_rows, width) / sizeof(int), "hipMalloc(gathered ids)");
            alloc(nb->frame, height * width * 4, "hipMalloc(frame)");
            if (m_out_half) {
                alloc(nb->frame16, height * width * 4, "hipMalloc(frame f16)");
            }
        }
    } catch (...) {
        ReleaseBuffers(*nb);
        throw;
    }
    if (m_buf) {
        if (!SyncAll()) {
            ReleaseBuffers(*nb);
            throw std::runtime_error("Configure: the devices did not finish earlier work");
        }
        ReleaseBuffers(*m_buf);
    }
    m_buf = std::move(nb);
    for (std::size_t i = 0; i < bands; ++i) {
        m_slots[i]->row_begin = split.RowBegin(i);
        m_slots[i]->row_count = split.RowCount(i);
    }
    m_band_rows = band_rows;
    m_width = width;
    m_height = height;
}

// On an exception mid-frame, copies already queued may still target the caller's host
// buffers: wait for every stream used (ignoring their errors) before the error propagates. Bounded
// (comm.h): false when a stream did not drain within the comm timeout.
bool Renderer::SyncAll() noexcept {
    const double t = CommTimeoutSeconds();
    bool ok = true;
    for (auto& sp : m_slots) {
        (void)hipSetDevice(sp->device);
        for (hipStream_t st : {sp->stream, sp->copy_in, sp->copy_out}) {
            if (st != nullptr && ok && !StreamDrain(st, t)) {
                ok = false;
            }
        }
    }
    return ok;
}

void Renderer::Render(const void* host_offsets, void* host_rgba) {
    if (!configured()) {
        throw std::runtime_error("Renderer used before Configure()");
    }
    int prev = -1;
    (void)hipGetDevice(&prev);
    try {
        if (m_slots.size() == 1 && m_gather_mode != GatherMode::kRccl && E2eChunks() > 1 &&
            m_height >= 2 * E2eChunks()) {
            RenderPipelined(host_offsets, host_rgba, E2eChunks());
        } else {
            RenderBands(host_offsets, host_rgba);
        }
    } catch (...) {
        // A failed gather may leave RCCL kernels waiting on peers: abort the communicators first
        // (their kernels exit, the streams drain); the model's later renders then fail loudly.
        if (!m_comms.empty()) {
            CommAbortAll(m_comms);
            m_comms_aborted = true;
        }
        (void)SyncAll();
        if (prev >= 0) {
            (void)hipSetDevice(prev);
        }
        throw;
    }
    if (prev >= 0) {
        (void)hipSetDevice(prev);
    }
}

// Copies band i's rows between a host frame (row_bytes per frame row) and a band-local device
// buffer: interleaved bands move one 16-row tile row per copy, contiguous bands one copy.
void Renderer::CopyBandRows(std::size_t i, const unsigned char* host, std::size_t row_bytes, unsigned char* dev,
                            hipMemcpyKind kind, bool to_host, hipStream_t stream) const {
    const Slot& s = *m_slots[i];
    const std::size_t interleave = m_interleaved && m_slots.size() > 1 ? m_slots.size() : 1;
    const std::size_t step = interleave > 1 ? static_cast<std::size_t>(kCullTileRows) : s.row_count;
    for (std::size_t l = 0; l < s.row_count; l += step) {
        const std::size_t n = std::min(step, s.row_count - l);
        const std::size_t fr = BandFrameRow(s.row_begin, interleave, l);
        unsigned char* h = const_cast<unsigned char*>(host) + fr * row_bytes;
        if (to_host) {
            HipCheck(hipMemcpyAsync(h, dev + l * row_bytes, n * row_bytes, kind, stream), "hipMemcpyAsync(band rows D2H)");
        } else {
            HipCheck(hipMemcpyAsync(dev + l * row_bytes, h, n * row_bytes, kind, stream), "hipMemcpyAsync(band rows H2D)");
        }
    }
}

// One band per device (module doc): band offsets in, hit ids traced, gathered to the first device,
// shaded there and copied out; "direct": every device shades its own rows and copies them out.
void Renderer::RenderBands(const void* host_offsets, void* host_rgba) {
    Buffers& b = *m_buf;
    const std::size_t w = m_width, h = m_height, P = m_slots.size();
    const std::size_t in_elem = m_in_half ? 2 : 4, out_elem = m_out_half ? 2 : 4;
    const auto* in_bytes = static_cast<const unsigned char*>(host_offsets);
    auto* out_bytes = static_cast<unsigned char*>(host_rgba);
    const std::size_t interleave = m_interleaved && P > 1 ? P : 1;
    const bool direct = (P == 1 && m_gather_mode != GatherMode::kRccl) || m_gather_mode == GatherMode::kDirect;
    if (m_comms_aborted) {
        throw std::runtime_error("RCCL communicators were aborted after an earlier failure; create the model again");
    }
    for (std::size_t i = 0; i < P; ++i) {
        Slot& s = *m_slots[i];
        DeviceGuard guard(s.device);
        if (s.row_count != 0) {
            auto* dst = m_in_half ? reinterpret_cast<unsigned char*>(b.offsets16[i])
                                  : reinterpret_cast<unsigned char*>(b.offsets[i]);
            CopyBandRows(i, in_bytes, w * 2 * in_elem, dst, hipMemcpyHostToDevice, false, s.stream);
            if (m_in_half) {
                HipCheck(LaunchHalfToFloat(b.offsets16[i], b.offsets[i], s.row_count * w * 2, s.stream),
                         "offsets f16 -> f32");
            }
        }
        s.scene->Prepare(w, h, s.stream);
        if (direct) {
            s.scene->Trace(b.offsets[i], b.rgba[i], s.row_begin, s.row_count, m_variant, s.stream, nullptr, interleave);
            auto* src = reinterpret_cast<unsigned char*>(b.rgba[i]);
            if (m_out_half) {
                HipCheck(LaunchFloatToHalf(b.rgba[i], b.rgba16[i], s.row_count * w * 4, s.stream),
                         "framebuffer f32 -> f16");
                src = reinterpret_cast<unsigned char*>(b.rgba16[i]);
            }
            CopyBandRows(i, out_bytes, w * 4 * out_elem, src, hipMemcpyDeviceToHost, true, s.stream);
        } else {
            s.scene->Trace(b.offsets[i], nullptr, s.row_begin, s.row_count, m_variant, s.stream, b.ids[i], interleave,
                           m_id_planes);
        }
    }
    if (!direct) {
        Slot& root = *m_slots.front();
        {
            DeviceGuard guard(root.device);  // the frame's offsets for shading
            void* dst = m_in_half ? static_cast<void*>(b.full16) : static_cast<void*>(b.full);
            HipCheck(hipMemcpyAsync(dst, in_bytes, h * w * 2 * in_elem, hipMemcpyHostToDevice, root.stream),
                     "hipMemcpyAsync(frame offsets H2D)");
            if (m_in_half) {
                HipCheck(LaunchHalfToFloat(b.full16, b.full, h * w * 2, root.stream), "offsets f16 -> f32");
            }
        }
        if (m_gather_mode == GatherMode::kRccl) {
            // Equal-size id bands (buffer rows each) gathered to the first device over xGMI, one
            // group; nonblocking communicators, so the gathers are on the streams once they settle.
            NcclCheck(ncclGroupStart(), "ncclGroupStart");
            ncclResult_t first = ncclSuccess;
            for (std::size_t i = 0; i < P; ++i) {
                Slot& s = *m_slots[i];
                const ncclResult_t r = ncclGather(b.ids[i], i == 0 ? b.gather : nullptr, BandIdBytes(m_band_rows, w), ncclUint8, 0,
                                                  static_cast<ncclComm_t>(m_comms[i]), s.stream);
                if (r != ncclSuccess && r != ncclInProgress && first == ncclSuccess) {
                    first = r;
                }
            }
            const ncclResult_t end = ncclGroupEnd();
            NcclCheck(first, "ncclGather");
            NcclCheck(end, "ncclGroupEnd (gather)", true);
            CommSettle(m_comms.data(), m_comms.size(), "gather enqueue");
        } else {
            // The same gather as device copies into the root's buffer (band i at i x buffer rows);
            // the root's stream then waits for every band's copy (an event per band).
            for (std::size_t i = 0; i < P; ++i) {
                Slot& s = *m_slots[i];
                DeviceGuard guard(s.device);
                HipCheck(hipMemcpyPeerAsync(reinterpret_cast<unsigned char*>(b.gather) + i * BandIdBytes(m_band_rows, w),
                                            root.device, b.ids[i], s.device, BandIdBytes(m_band_rows, w), s.stream),
                         "hipMemcpyPeerAsync(band gather)");
                if (i != 0) {
                    if (s.traced.empty()) {
                        hipEvent_t e = nullptr;
                        HipCheck(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate(band gather)");
                        s.traced.push_back(e);
                    }
                    HipCheck(hipEventRecord(s.traced[0], s.stream), "hipEventRecord(band gather)");
                    DeviceGuard root_guard(root.device);
                    HipCheck(hipStreamWaitEvent(root.stream, s.traced[0], 0), "hipStreamWaitEvent(band gather)");
                }
            }
        }
        DeviceGuard guard(root.device);
        root.scene->Shade(b.full, b.gather, b.frame, 0, h, root.stream, 1, m_band_rows, interleave > 1 ? P : 0, 0,
                          m_id_planes);
        const void* src = b.frame;
        if (m_out_half) {
            HipCheck(LaunchFloatToHalf(b.frame, b.frame16, h * w * 4, root.stream), "framebuffer f32 -> f16");
            src = b.frame16;
        }
        HipCheck(hipMemcpyAsync(out_bytes, src, h * w * 4 * out_elem, hipMemcpyDeviceToHost, root.stream),
                 "hipMemcpyAsync(frame D2H)");
    }
    // Every device's work done: polled with a deadline and the communicators' async errors (a
    // peer that stopped becomes an error here, not a hang).
    for (auto& sp : m_slots) {
        DeviceGuard guard(sp->device);
        if (sp->done == nullptr) {
            HipCheck(hipEventCreateWithFlags(&sp->done, hipEventDisableTiming), "hipEventCreate(done)");
        }
        HipCheck(hipEventRecord(sp->done, sp->stream), "hipEventRecord(done)");
    }
    for (auto& sp : m_slots) {
        DeviceGuard guard(sp->device);
        CommWaitEvent(sp->done, m_comms.data(), m_comms.size(), "render");
    }
}

// One device: the frame in row chunks, H2D of chunk c+1 and D2H of chunk c-1 overlapping the
// trace of chunk c (three streams, event-ordered). Every chunk is an ordinary band trace of
// the same prepared frame, so the image is bit-identical to the unchunked render.
void Renderer::RenderPipelined(const void* host_offsets, void* host_rgba, std::size_t chunks) {
    Slot& s = *m_slots.front();
    Buffers& b = *m_buf;
    DeviceGuard guard(s.device);
    const std::size_t w = m_width, h = m_height;
    const std::size_t in_elem = m_in_half ? 2 : 4, out_elem = m_out_half ? 2 : 4;
    const auto* in_bytes = static_cast<const unsigned char*>(host_offsets);
    auto* out_bytes = static_cast<unsigned char*>(host_rgba);
    if (s.copy_in == nullptr) {
        HipCheck(hipStreamCreateWithFlags(&s.copy_in, hipStreamNonBlocking), "hipStreamCreate(copy in)");
        HipCheck(hipStreamCreateWithFlags(&s.copy_out, hipStreamNonBlocking), "hipStreamCreate(copy out)");
    }
    while (s.in_done.size() < chunks) {
        hipEvent_t e0 = nullptr, e1 = nullptr;
        HipCheck(hipEventCreateWithFlags(&e0, hipEventDisableTiming), "hipEventCreate(chunk)");
        HipCheck(hipEventCreateWithFlags(&e1, hipEventDisableTiming), "hipEventCreate(chunk)");
        s.in_done.push_back(e0);
        s.traced.push_back(e1);
    }
    float* offsets = b.offsets[0];
    float* rgba = b.rgba[0];
    const std::size_t rows = (h + chunks - 1) / chunks;
    s.scene->Prepare(w, h, s.stream);
    // Direct output (f32 output images; env SRT_E2E_DIRECT=0: off): the trace stores each chunk's
    // framebuffer rows straight into the page-locked host image through its device mapping -- the stores
    // cross PCIe from the CUs while the copy engine moves the next chunk's offsets in, instead of both
    // directions queuing on copy engines (pinned H2D + D2H at once measured 57 GB/s together, no faster
    // than one after the other). 1080p C3: 1.41 -> 0.89 ms per frame on a box whose copy path read
    // 1.41 (another box: 0.82 with copies); bit-identical (test_ml_pipelined_chunks_bitwise).
    float* direct = nullptr;
    {
        static const bool want = [] {
            const char* v = std::getenv("SRT_E2E_DIRECT");
            return v == nullptr || std::strcmp(v, "0") != 0;
        }();
        void* dp = nullptr;
        if (want && !m_out_half && hipHostGetDevicePointer(&dp, host_rgba, 0) == hipSuccess && dp != nullptr) {
            direct = static_cast<float*>(dp);
        }
        (void)hipGetLastError();  // (a pageable image: no mapping, the copy path)
    }
    for (std::size_t c = 0; c < chunks; ++c) {
        const std::size_t r0 = c * rows;
        if (r0 >= h) {
            break;
        }
        const std::size_t n = std::min(rows, h - r0);
        const std::size_t count = n * w * 2;
        void* dst = m_in_half ? static_cast<void*>(b.offsets16[0] + r0 * w * 2) : static_cast<void*>(offsets + r0 * w * 2);
        HipCheck(hipMemcpyAsync(dst, in_bytes + r0 * w * 2 * in_elem, count * in_elem, hipMemcpyHostToDevice, s.copy_in),
                 "hipMemcpyAsync(offsets chunk H2D)");
        HipCheck(hipEventRecord(s.in_done[c], s.copy_in), "hipEventRecord(chunk in)");
        HipCheck(hipStreamWaitEvent(s.stream, s.in_done[c], 0), "hipStreamWaitEvent(chunk in)");
        if (m_in_half) {
            HipCheck(LaunchHalfToFloat(b.offsets16[0] + r0 * w * 2, offsets + r0 * w * 2, count, s.stream),
                     "offsets f16 -> f32");
        }
        if (direct != nullptr) {
            s.scene->Trace(offsets + r0 * w * 2, direct + r0 * w * 4, r0, n, m_variant, s.stream);
            continue;
        }
        s.scene->Trace(offsets + r0 * w * 2, rgba + r0 * w * 4, r0, n, m_variant, s.stream);
        if (m_out_half) {
            HipCheck(LaunchFloatToHalf(rgba + r0 * w * 4, b.rgba16[0] + r0 * w * 4, n * w * 4, s.stream),
                     "framebuffer f32 -> f16");
        }
        HipCheck(hipEventRecord(s.traced[c], s.stream), "hipEventRecord(chunk traced)");
        HipCheck(hipStreamWaitEvent(s.copy_out, s.traced[c], 0), "hipStreamWaitEvent(chunk traced)");
        const void* src = m_out_half ? static_cast<const void*>(b.rgba16[0] + r0 * w * 4)
                                     : static_cast<const void*>(rgba + r0 * w * 4);
        HipCheck(hipMemcpyAsync(out_bytes + r0 * w * 4 * out_elem, src, n * w * 4 * out_elem, hipMemcpyDeviceToHost,
                                s.copy_out),
                 "hipMemcpyAsync(frame chunk D2H)");
    }
    HipCheck(hipStreamSynchronize(s.copy_out), "render (copy out)");
    HipCheck(hipStreamSynchronize(s.stream), "render");
}

}  // namespace srt
