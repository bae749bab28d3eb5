// Frame engine: a stream of frames rendered over one or more GPUs (SURVEY.md section 8 rows a9-a13,
// (e)), the native counterpart of what bench.py and a multi-GPU host renderer drive.
//
// A run is a sequence of *batches* of F frames. Each local device keeps Q frame queues (its own
// DeviceScene, HIP stream and buffers each); batch b runs on queue b % Q of every device, so Q
// batches are in flight per device.
//
// Split "bands" over P devices (BASELINE config C4): every frame is cut into P row bands -- the
// frame's 16-row tile rows dealt round-robin (interleaved, default) or P contiguous blocks --,
// device d traces band d of the batch's F frames (hit ids only, 4 B per pixel), the bands move to
// the frames' compositors over RCCL, and each compositor shades its frames from the gathered ids
// (deferred shading, bit-identical to the fused trace). Exchange patterns:
//   kAllToAll       frame f of a batch is composited on device f % P: the batch's P gathers
//                   (one per compositor) are fused into one group of ncclSend / ncclRecv, so every
//                   directed xGMI link carries 1/P of the payload;
//   kRotatingGather the whole batch is gathered to device b % P (one gather per batch);
//   kRootGather     everything to device 0;
//   kShare          frame f of a batch is composited on device c = f % P (as all-to-all), which
//                   traces `share` (k) of every k + P - 1 tile rows of it itself -- straight into the
//                   frame as RGBA -- while every other device traces one tile row of each such cycle
//                   (its class) and sends its ids: the exchange and the deferred shading shrink to
//                   (P - 1) / (k + P - 1) of a frame (1080p: k = 32, P = 2: 1/33; P = 8: 7/39), and
//                   every batch loads every device alike (a compositor per batch, rotating, left
//                   the other devices idle behind its long trace unless P batches were in flight).
// P == 1 traces and shades in one kernel (RGBA), no exchange.
// Split "frames": every device renders whole frames of its own (no exchange; weak scaling).
//
// Devices are either all in this process (one worker thread per device, one nonblocking RCCL
// communicator per device from one group of ncclCommInitRankConfig; a repeated device -- "fake
// devices" on a one-GPU box -- or SRT_GATHER=copy exchanges by device copies instead), or one per
// process (rank mode: ncclCommInitRankConfig with a unique id the ranks share, one rank per GPU as
// torch.distributed.run launches them).
//
// Failures end in an error, never a hang (comm.h): every wait behind RCCL polls with a deadline
// (SRT_COMM_TIMEOUT_S), a worker's failure or a stall of every device aborts the communicators
// (ncclCommAbort) and Run() throws the first error; the engine then refuses further work.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "comm.h"
#include "renderer.h"
#include "scene.h"

namespace srt {

struct EngineOptions {
    enum Split { kBands = 0, kFrames = 1 };
    enum Exchange { kAllToAll = 0, kRotatingGather = 1, kRootGather = 2, kShare = 3 };
    int variant = 2;           // render.h TraceVariant (kTraceCull)
    std::size_t queues = 2;    // batches in flight per device
    std::size_t batch = 16;    // frames per batch
    bool interleaved = true;   // bands: tile rows dealt round-robin (else contiguous blocks)
    // Contiguous bands (interleaved false) with kAllToAll: device p traces band (p + c) % P of a frame
    // composited on device c, so over any P consecutive frames every device traces every band once
    // (even load whatever the scene's density profile) while each band stays one contiguous block of
    // rows, which the band record pass's block skip needs (render.h CullBins::block_ext).
    bool rotate = false;
    int exchange = kAllToAll;  // bands at P > 1
    int split = kBands;
    // Measurement only: one rank of a world-device job with no peers -- the rank's whole stream
    // (band traces, its share of the compositing) without the exchange, which is skipped (its
    // composited frames are then garbage). The per-rank GPU time of the multi-GPU pipeline on one GPU.
    bool simulate = false;
    // Frames per trace launch (a batch is traced in ceil(batch / launch) launch sets of four
    // kernels; more than render.h kMaxBatch frames take their parameters from a device table).
    // 0: env SRT_LAUNCH_FRAMES, else the default: kMaxBatch for whole frames (larger launches of
    // full frames measured slower: C3 114.4 / 107.0 / 101.9 / 105.1 Grays/s at 8 / 16 / 32 / 64),
    // FrameEngine::kDefaultBandLaunch for bands at P > 1 (per-rank time at P = 8: 6.05 / 5.81 /
    // 5.84 / 5.66 us per frame).
    std::size_t launch = 0;
    // Test / measurement: one device, the bands path with the frame's ids sent to itself over a
    // one-rank RCCL communicator (ncclSend / ncclRecv to self) -- the real exchange, its waits and
    // its abort path on a one-GPU box. Frames are bit-identical to the fused trace.
    bool rccl_self = false;
    // kShare: the compositor's tile rows per cycle (k above, a power of two; 0: ShareAuto).
    std::size_t share = 0;
    // Rotated bands over two devices: rows of the compositor's own band 0 (0: env SRT_ROTATE_OWN per cent
    // if set, else -- RCCL between distinct devices -- derived from the link measured at creation
    // (RotateSplitForLink), else 80 % of the frame).
    std::size_t own_rows = 0;
};

// kShare's default k for an H-row frame over P devices: the largest power of two <= 32 with
// k + P - 1 <= the frame's tile rows (engine.cpp).
std::size_t ShareAuto(std::size_t height, std::size_t world);

// Rows of the compositor's own band under rotated all-to-all over two devices without a measured
// link: env SRT_ROTATE_OWN per cent (an integer in 1..99, else std::runtime_error), default 80, rounded
// to tile rows (engine.cpp).
std::size_t RotateOwnRows(std::size_t height);
long RotateOwnPercent();  // env SRT_ROTATE_OWN, validated; 0 when unset
// The two-device split for a link of `link_gbs` GB/s per direction, a one-GPU frame time of `frame_us`
// and an exchange payload of `bytes_per_pixel`: the smallest own band (tile rows, >= H / 2) whose link
// time stays within 80 % of the GPU time per frame of the job (engine.cpp).
std::size_t RotateSplitForLink(std::size_t height, std::size_t width, double link_gbs, double frame_us,
                               double bytes_per_pixel);

// Row bands of an H-row frame over P devices (interleaved or contiguous), the layout every
// exchange path and the shading kernel agree on.
struct BandSplit {
    std::size_t height = 0, bands = 1;
    bool interleaved = true;
    std::size_t first_sent = 0;  // bands below it never travel (kShare: the compositor's own classes)
    // Contiguous bands: rows of band 0 (0: every band ceil(H / P) rows, the last one shorter); the
    // other bands split the rest evenly. Rotated all-to-all over 2 devices, where band 0 is always the
    // compositor's own (FrameEngine: the one link carries the other band of every frame).
    std::size_t first_rows = 0;
    static BandSplit Make(std::size_t height, std::size_t bands, bool interleaved);
    std::size_t RowBegin(std::size_t band) const;  // first frame row (interleaved: band * 16)
    std::size_t RowCount(std::size_t band) const;  // rows of the band
    std::size_t BufferRows() const;                // rows of every sent band's (padded) buffer: the largest
    std::size_t Interleave() const { return interleaved && bands > 1 ? bands : 1; }
    std::size_t FrameRow(std::size_t band, std::size_t local) const;
};

// The engine's band split for P = `world` devices (bands: P bands, kShare share + P - 1 classes; rotated
// over two devices band 0 takes own_rows, 0: RotateOwnRows) -- shared with the host self-test.
BandSplit EngineSplit(std::size_t height, std::size_t world, bool bands, bool interleaved, bool rotate,
                      std::size_t share, std::size_t own_rows);

// Which device composites frame f of batch b, and that frame's slot among the device's frames.
struct ExchangePlan {
    std::size_t bands = 1, batch = 1;  // bands: the devices (P)
    int exchange = EngineOptions::kAllToAll;
    std::size_t Compositor(std::size_t batch_index, std::size_t f) const;
    std::size_t Slot(std::size_t f) const;                                      // index among its compositor's frames
    std::size_t FramesFor(std::size_t batch_index, std::size_t compositor) const;  // frames composited there
    std::size_t MaxFramesPerCompositor() const;
    bool rotate = false;  // EngineOptions::rotate (kAllToAll over contiguous bands)
    // Slot of device p's ids in compositor c's receive buffer (kShare: the senders in class order;
    // rotate: the band p traces for c, so the buffer is band-major in band order).
    std::size_t RecvSlot(std::size_t c, std::size_t p) const;
    // The band device p traces of a frame composited on device c (rotate: (p + c) % P, else p).
    std::size_t BandOf(std::size_t p, std::size_t c) const { return rotate ? (p + c) % bands : p; }
    // Frames of a batch dealt to compositors round-robin (kAllToAll, kShare), not whole batches.
    bool PerFrame() const { return exchange == EngineOptions::kAllToAll || exchange == EngineOptions::kShare; }
};

// Host self-test of the exchange (no device): band_ids[d] = device d's traced ids of the batch's F
// frames, frame-major (F x buffer rows x width int32: of frame f its band, plan.BandOf(d, compositor
// of f) under rotate). Returns, for compositor c, its receive buffer exactly as the device path lays
// it out: [P][FramesFor(b, c)][buffer rows][W], device d's frames at slot plan.RecvSlot(c, d).
std::vector<std::vector<int>> ExchangeOnHost(const BandSplit& split, const ExchangePlan& plan, std::size_t width,
                                             std::size_t batch_index, const std::vector<std::vector<int>>& band_ids);

class FrameEngine {
public:
    // All devices in this process.
    FrameEngine(const Scene& scene, const std::vector<int>& devices, std::size_t width, std::size_t height,
                const EngineOptions& options);
    // One device of a `world`-device job, this process being `rank` (unique_id: 128 bytes from
    // UniqueId() on rank 0, shared by every rank; every rank constructs concurrently).
    FrameEngine(const Scene& scene, int device, int rank, int world, const void* unique_id, std::size_t width,
                std::size_t height, const EngineOptions& options);
    ~FrameEngine();
    FrameEngine(const FrameEngine&) = delete;
    FrameEngine& operator=(const FrameEngine&) = delete;

    static void UniqueId(void* out128);
    // Host self-test of the worker pool's failure handling (no device): `workers` workers, worker
    // `failing` throws (mode Injection::kFail) or stalls (kStall) while every other worker waits
    // for a release only the abort gives. Returns the error Run() threw ("" if none), the seconds
    // it took and how many times the abort hook ran.
    static std::string PoolSelfTest(std::size_t workers, std::size_t failing, int mode, double timeout_s,
                                    double* elapsed_s, int* abort_calls);
    static constexpr std::size_t kDefaultBandLaunch = 64;

    // `count` full-frame sample-offset images (count x H x W x 2 floats, host), resident on every
    // local device from now on (each device keeps the frames and its band's rows of each); frame k
    // of a run reads input k % count. Bands at P > 1 with count > 1 need count % batch == 0 and
    // (all-to-all) batch % P == 0, so a compositor's frames read evenly strided inputs.
    void SetInputs(const float* host_offsets, std::size_t count);
    // Render `batches` batches (batch x frames each), continuing the frame sequence; returns when
    // every local device has finished.
    void Run(std::size_t batches);
    // The frames composited locally in each queue's last batch (the first `per_queue` of them),
    // compared bit for bit with a single-device full-frame render of their inputs. Returns the
    // number of mismatching frames; `checked` receives the number compared.
    std::size_t Verify(std::size_t* checked, std::size_t per_queue = 4);
    // Frame k (of the last Q batches) into host RGBA (H x W x 4 floats); false when frame k is not
    // resident on a local device (another rank composited it, or it is older).
    bool ReadFrame(std::size_t k, float* host_rgba);
    // Stage times of `launches` traces of `frames` frames each (1 .. batch; one launch per stage for
    // all of them) of local device `local`'s band, one launch in flight (HIP events bound to the
    // kernels' dispatches): mean ms per launch of tile info, record setup + bins + work list, trace.
    DeviceScene::StageTimes MeasureStages(std::size_t local, std::size_t launches, std::size_t frames = 1);

    // A failed run left a device worker stuck in a HIP call (GPU unresponsive): the worker still runs
    // inside this engine, so its owner must leak it instead of destroying it (srtEngineRelease).
    bool wedged() const { return m_wedged; }
    std::size_t devices() const { return m_world; }
    std::size_t local_devices() const { return m_dev.size(); }
    std::size_t frames_per_batch() const { return m_opt.batch; }
    std::size_t frames_rendered() const;  // this run's frames over all devices (frames split: x P)
    std::size_t band_rows(std::size_t local) const;
    std::size_t buffer_rows() const { return m_split.BufferRows(); }
    bool uses_rccl() const { return m_exchange && !m_copy && !m_opt.simulate && m_comms_made; }
    std::uint64_t triangles() const { return m_n; }
    // Bytes the devices exchange per frame (bands at P > 1), for the report.
    double exchange_bytes_per_frame() const;
    // The last run's exchange on local device `local`, timed by HIP events on its exchange stream
    // around each batch's send / receive group (RCCL) or copies (device copies): groups, mean ms per
    // group, and the bytes the device sent per group (to all peers).
    struct ExchangeStats {
        std::size_t groups = 0;
        double ms_mean = 0.0;
        double bytes_sent = 0.0;
    };
    ExchangeStats exchange_stats(std::size_t local) const;
    int id_planes() const { return m_id_planes; }  // exchange payload: packed ids' bit planes, -1 int32
    // The two-device split and where it came from (srtEngineSplit): own band rows (0: no two-device
    // rotated split), the band buffers' rows, the link measured at creation (GB/s per direction, 0: not
    // measured -- no RCCL), the one-GPU frame time measured for the split (us, 0: not measured).
    enum SplitSource { kSplitNone = 0, kSplitOption = 1, kSplitEnv = 2, kSplitLink = 3, kSplitDefault = 4 };
    struct SplitInfo {
        std::size_t own_rows = 0, buffer_rows = 0;
        double link_gbs = 0.0, frame_us = 0.0;
        int source = kSplitNone;
    };
    SplitInfo split_info() const;

private:
    struct Queue;
    struct Device;
    struct Pool;
    void Init(const Scene& scene, const std::vector<int>& devices);
    void Release() noexcept;
    void AllocateQueues();
    void AbortComms() noexcept;  // sets the abort flag, then ncclCommAbort under the exclusive lock
    void CheckUsable() const;    // throws once a run has failed
    void Inject(std::size_t local, std::size_t b);  // SRT_ENGINE_INJECT (comm.h)
    std::size_t FrameIndex(std::size_t local, std::size_t b, std::size_t f) const;  // frame of the sequence
    int* Ids(unsigned char* buf, std::size_t band_frame) const;  // band frame `band_frame` of an id buffer
    // A device's band in one role: bands / rotating / root have one role (its band); kShare has role 0
    // (compositor: k of every k + P - 1 tile rows, RGBA) and roles 1 .. P - 1 (sender of class
    // k + role - 1: one tile row per cycle, ids).
    struct Role {
        std::size_t row_begin = 0, rows = 0, pattern = 1;
        std::size_t input = 0;  // rows of the earlier roles (Device::band_in: per role, inputs x rows x W x 2)
    };
    std::size_t RoleOf(std::size_t local, std::size_t compositor) const;  // role for a frame composited there
    bool m_rotate = false;  // EngineOptions::rotate at P > 1: roles = the P contiguous bands, inputs from `full`
    void TracePhase(std::size_t local, std::size_t b);
    void TraceShare(std::size_t local, std::size_t b);  // kShare's trace: each frame in its compositor's pattern
    void TraceRotated(std::size_t local, std::size_t b);  // rotate: each frame's band by its compositor
    void ExchangePhase(std::size_t local, std::size_t b);  // RCCL: inside a group
    double SentBytes(std::size_t local, std::size_t b) const;  // ids device `local` sends for batch b
    void CopyPhase(std::size_t local, std::size_t b);      // device-copy exchange
    hipEvent_t* ExchangeEvents(std::size_t local);          // the next timing pair (a bounded ring)
    void AddExchangeTime(std::size_t local, std::size_t slot);  // wait for a pair, add its time
    void ShadePhase(std::size_t local, std::size_t b);
    void RunWorker(std::size_t local, std::size_t b0, std::size_t batches);
    void Barrier();
    const float* BandInput(std::size_t local, std::size_t k, std::size_t role = 0) const;
    const float* FullInput(std::size_t local, std::size_t k) const;
    std::size_t FrameFloats() const { return m_width * m_height * 2; }
    void PrimeSimulation();  // simulate: receive buffers hold real ids (the sender role's band)
    void Layout(std::size_t own_rows);  // m_split, m_band_id_bytes and every device's roles
    std::size_t SenderRole(std::size_t local) const;  // a role whose ids fit one band buffer
    void SettleSplit();      // after the communicators: link rate, derived / agreed two-device split
    double MeasureLink();    // GB/s per direction (RCCL send / receive groups), over every rank
    double MeasureFrameUs();  // one GPU's us per whole frame (8-frame traces), over every rank
    std::vector<double> MaxOverRanks(const std::vector<double>& v);  // rank mode: ncclAllReduce(max)
    int m_split_source = kSplitNone;
    double m_link_gbs = 0.0, m_frame_us = 0.0;

    EngineOptions m_opt;
    std::size_t m_width = 0, m_height = 0, m_world = 1, m_rank0 = 0;  // m_rank0: global index of local 0
    std::uint64_t m_n = 0;
    bool m_bands = true;       // bands split (at P > 1, or rccl_self: exchange + shading)
    bool m_exchange = false;   // bands with an exchange: P > 1, or the one-device RCCL self-exchange
    int m_id_planes = -1;          // exchange payload: packed ids with this many bit planes (render.h PackedIds), -1 int32
    std::size_t m_band_id_bytes = 0;  // one band frame of it
    bool m_comms_made = false; // RCCL communicators were created (uses_rccl after an abort too)
    bool m_copy = false;       // exchange by device copies (repeated device / SRT_GATHER=copy)
    bool m_defer_shade = false;  // env SRT_DEFER_SHADE=1 (measurement): whole frames as ids + a shading launch
    std::size_t m_share = 0;     // kShare: the compositor's tile rows per cycle (0: another exchange)
    BandSplit m_split;
    ExchangePlan m_plan;
    std::vector<std::unique_ptr<Device>> m_dev;
    std::vector<void*> m_comms;  // ncclComm_t per local device (nonblocking; empty once aborted)
    std::unique_ptr<CommCtl> m_ctl;  // abort flag, progress counter, communicator lock (comm.h)
    Injection m_inject;
    std::string m_failed;      // the first error of a failed run (the engine is then unusable)
    bool m_wedged = false;     // a worker never returned from a failed run (its pool is leaked)
    std::unique_ptr<Pool> m_pool;
    std::size_t m_inputs = 0;
    std::size_t m_next_batch = 0;  // batches issued so far (the frame sequence continues across runs)
    std::size_t m_run_batches = 0;
    std::unique_ptr<Scene> m_scene;  // for Verify's reference renders
};

}  // namespace srt
