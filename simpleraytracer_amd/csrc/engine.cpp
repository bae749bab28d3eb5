#include "engine.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <functional>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>

#include "comm.h"
#include "render.h"

namespace srt {
namespace {

template <class T>
T* DeviceAlloc(std::size_t count, const char* what) {
    void* p = nullptr;
    HipCheck(hipMalloc(&p, (count == 0 ? 1 : count) * sizeof(T)), what);
    return static_cast<T*>(p);
}

bool GatherByCopies(const std::vector<int>& devices) {
    const char* v = std::getenv("SRT_GATHER");
    if (v != nullptr && std::strcmp(v, "copy") == 0) {
        return true;
    }
    for (std::size_t i = 0; i < devices.size(); ++i) {
        for (std::size_t j = 0; j < i; ++j) {
            if (devices[i] == devices[j]) {
                return true;  // one device twice: no RCCL communicator (the "fake devices" rehearsal)
            }
        }
    }
    return false;
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// The share exchange's default k: the largest power of two <= 32 whose cycle of k + P - 1 tile rows
// still fits the frame (every sender traces at least one tile row). Measured (tools/rank_sim.py,
// 1080p, balanced batch counts; profiles/r04/share/): the larger k, the fewer rows take the ids path
// (trace to ids, exchange, deferred shading) instead of the fused trace-and-shade, so the GPU time
// per frame falls -- P = 2: k = 4 12.0, 16 10.9 us; P = 4: 8.2 all-to-all, 6.7 at k = 32; P = 8:
// 5.3 all-to-all, 4.6 at 16, 4.4 at 32 -- and so do the bytes on the links. The price is latency:
// the compositor traces k / (k + P - 1) of each of its frames.
std::size_t ShareAuto(std::size_t height, std::size_t world) {
    const std::size_t tile_rows = (height + kCullTileRows - 1) / kCullTileRows;
    std::size_t k = 32;
    while (k > 1 && k + world - 1 > tile_rows) {
        k /= 2;
    }
    return k;
}

// Rows of the compositor's own band under rotated all-to-all over two devices (env SRT_ROTATE_OWN: per
// cent of the frame, default 80; 50 = even halves), rounded to whole 16-row tile rows. Even halves send
// half of every frame's ids over the one link: 1.1 MB per frame of the job each way at 1080p, 17 us at an
// assumed 64 GB/s against 11 us of GPU time (rank simulation) -- link-bound below one GPU; a fifth
// (216 of 1080 rows) cuts that to 7.2 us (GPU-bound down to ~45 GB/s) and the compositor's deferred
// shading with it.
long RotateOwnPercent() {
    const char* v = std::getenv("SRT_ROTATE_OWN");
    if (v == nullptr || *v == '\0') {
        return 0;
    }
    char* end = nullptr;
    errno = 0;
    const long pct = std::strtol(v, &end, 10);
    if (errno != 0 || end == v || *end != '\0' || pct < 1 || pct > 99 || (*v != '+' && (*v < '0' || *v > '9'))) {
        throw std::runtime_error(std::string("SRT_ROTATE_OWN must be an integer per cent in 1..99, got '") + v + "'");
    }
    return pct;
}

std::size_t RotateOwnRowsAt(std::size_t height, long pct) {
    const std::size_t t = static_cast<std::size_t>(kCullTileRows);
    std::size_t rows = (height * static_cast<std::size_t>(pct) + 50) / 100;
    rows = height > 2 * t ? (rows + t / 2) / t * t : rows;
    return std::max<std::size_t>(1, std::min(rows, height > 1 ? height - 1 : 1));
}

std::size_t RotateOwnRows(std::size_t height) {
    const long pct = RotateOwnPercent();
    return RotateOwnRowsAt(height, pct == 0 ? 80 : pct);
}

// The two-device split from a measured link. Per frame of the job, each
// direction of the one link carries the sent band of every second frame: (H - r) W b / 2 bytes at
// `link_gbs`; the GPUs spend frame_us (0.553 + 0.25 (H - r) / H) per frame of the job -- the rank
// simulation's P = 2 times over the own share r / H (profiles/r05/rank_sim/p2_own_split.txt: 11.49 /
// 10.36 / 10.22 / 10.12 us at 50 / 75 / 80 / 85 %, one GPU 16.96 us), the deferred shading of the sent
// rows being the part that does not halve. The smallest own band (the most even tiling) whose link
// time stays within 80 % of that GPU time, so the link is not the bound; the largest own band (at most
// one tile row sent) when no split reaches it.
std::size_t RotateSplitForLink(std::size_t height, std::size_t width, double link_gbs, double frame_us,
                               double bytes_per_pixel) {
    const std::size_t t = static_cast<std::size_t>(kCullTileRows);
    if (height < 2) {
        return 1;
    }
    const std::size_t hi = height > 2 * t ? (height - 1) / t * t : height - 1;  // whole tile rows, one row at least sent
    if (!(link_gbs > 0.0) || !(frame_us > 0.0) || !(bytes_per_pixel > 0.0)) {
        return hi;
    }
    const double H = static_cast<double>(height), W = static_cast<double>(width);
    std::size_t r = (height + 1) / 2;
    r = height > 2 * t ? (r + t - 1) / t * t : r;
    for (; r <= hi; r += height > 2 * t ? t : 1) {
        const double sent = H - static_cast<double>(r);
        const double link_us = sent * W * bytes_per_pixel / 2.0 / (link_gbs * 1e3);
        const double gpu_us = frame_us * (0.553 + 0.25 * sent / H);
        if (link_us <= 0.8 * gpu_us) {
            return std::min(r, hi);
        }
    }
    return hi;
}

BandSplit EngineSplit(std::size_t height, std::size_t world, bool bands, bool interleaved, bool rotate,
                      std::size_t share, std::size_t own_rows) {
    BandSplit s = BandSplit::Make(height, bands ? (share != 0 ? share + world - 1 : world) : 1, interleaved);
    s.first_sent = share;
    if (bands && rotate && world == 2 && !interleaved) {
        // Two devices: band 0 (the compositor's own: BandOf(c, c) = 0) takes own_rows of the frame. Per
        // pair of frames each device still traces one band 0 and one band 1 (one frame's work), but only
        // band 1 crosses the single link and waits for the deferred shading.
        s.first_rows = own_rows != 0 ? std::min(own_rows, height > 1 ? height - 1 : 1) : RotateOwnRows(height);
        s.first_sent = 1;
    }
    return s;
}

// Band split and exchange plan (pure index math; shared with the host self-test).

BandSplit BandSplit::Make(std::size_t height, std::size_t bands, bool interleaved) {
    BandSplit s;
    s.height = height;
    s.bands = bands == 0 ? 1 : bands;
    s.interleaved = interleaved;
    return s;
}

namespace {
// Contiguous bands: band 0's rows and every later band's (the last one shorter).
void ContiguousRows(const BandSplit& s, std::size_t& first, std::size_t& step) {
    if (s.first_rows != 0 && s.bands > 1) {
        first = std::min(s.first_rows, s.height);
        step = (s.height - first + s.bands - 2) / (s.bands - 1);
    } else {
        first = step = (s.height + s.bands - 1) / s.bands;
    }
}
}  // namespace

std::size_t BandSplit::RowBegin(std::size_t band) const {
    if (bands == 1) {
        return 0;
    }
    if (interleaved) {
        return std::min(height, band * static_cast<std::size_t>(kCullTileRows));
    }
    std::size_t first = 0, step = 0;
    ContiguousRows(*this, first, step);
    return band == 0 ? 0 : std::min(height, first + (band - 1) * step);
}

std::size_t BandSplit::RowCount(std::size_t band) const {
    if (bands == 1) {
        return height;
    }
    if (interleaved) {
        return InterleavedBandRows(height, bands, band);
    }
    std::size_t first = 0, step = 0;
    ContiguousRows(*this, first, step);
    return std::min(height, first + band * step) - RowBegin(band);
}

std::size_t BandSplit::BufferRows() const {
    if (bands == 1) {
        return height;
    }
    if (!interleaved) {  // the largest band that travels
        std::size_t rows = 0;
        for (std::size_t j = first_sent; j < bands; ++j) {
            rows = std::max(rows, RowCount(j));
        }
        return std::max<std::size_t>(rows, 1);
    }
    // The largest band that travels (interleaved bands need not shrink with the index: the one
    // holding a partial last tile row may be shorter than the next). kShare: the sender classes only
    // -- sizing by class 0 padded every sender's buffer to 2 tile rows at P = 8 (1080p) for 1 traced.
    std::size_t rows = 0;
    for (std::size_t j = first_sent; j < bands; ++j) {
        rows = std::max(rows, InterleavedBandRows(height, bands, j));
    }
    return std::max<std::size_t>(rows, 1);
}

std::size_t BandSplit::FrameRow(std::size_t band, std::size_t local) const {
    return BandFrameRow(RowBegin(band), Interleave(), local);
}

std::size_t ExchangePlan::Compositor(std::size_t batch_index, std::size_t f) const {
    switch (exchange) {
        case EngineOptions::kRotatingGather:
            return batch_index % bands;
        case EngineOptions::kRootGather:
            return 0;
        default:
            return f % bands;
    }
}

std::size_t ExchangePlan::Slot(std::size_t f) const {
    return PerFrame() ? f / bands : f;
}

std::size_t ExchangePlan::FramesFor(std::size_t batch_index, std::size_t compositor) const {
    switch (exchange) {
        case EngineOptions::kRotatingGather:
            return compositor == batch_index % bands ? batch : 0;
        case EngineOptions::kRootGather:
            return compositor == 0 ? batch : 0;
        default:
            return compositor < batch ? (batch - compositor + bands - 1) / bands : 0;
    }
}

std::size_t ExchangePlan::MaxFramesPerCompositor() const {
    return PerFrame() ? (batch + bands - 1) / bands : batch;
}

std::size_t ExchangePlan::RecvSlot(std::size_t c, std::size_t p) const {
    if (rotate) {
        return BandOf(p, c);
    }
    return exchange == EngineOptions::kShare ? (p + bands - c - 1) % bands : p;
}

namespace {
// Band frame index of compositor c's slot j in a device's send buffer: all-to-all keeps one region
// of MaxFramesPerCompositor frames per compositor; the gathers send everything to one.
std::size_t SendFrames(const ExchangePlan& plan, std::size_t c, std::size_t j) {
    const std::size_t region = plan.PerFrame() ? c * plan.MaxFramesPerCompositor() : 0;
    return region + j;
}
std::size_t SendPixels(const ExchangePlan& plan, std::size_t c, std::size_t j, std::size_t band_pixels) {
    return SendFrames(plan, c, j) * band_pixels;
}
}  // namespace

std::vector<std::vector<int>> ExchangeOnHost(const BandSplit& split, const ExchangePlan& plan, std::size_t width,
                                             std::size_t batch_index, const std::vector<std::vector<int>>& band_ids) {
    // kShare: split holds the share + P - 1 classes, every band buffer one class (the sender's).
    const std::size_t P = plan.bands, B = split.BufferRows(), F = plan.batch;
    const std::size_t band_pixels = B * width;
    if (band_ids.size() != P) {
        throw std::runtime_error("ExchangeOnHost: one id buffer per band");
    }
    for (const auto& ids : band_ids) {
        if (ids.size() != F * band_pixels) {
            throw std::runtime_error("ExchangeOnHost: id buffers must be frames x buffer rows x width");
        }
    }
    std::vector<std::vector<int>> recv(P);
    for (std::size_t c = 0; c < P; ++c) {
        const std::size_t n = plan.FramesFor(batch_index, c);
        recv[c].assign(P * n * band_pixels, -1);
        // What device d sends to c (its send buffer region in SendPixels order), landing at region
        // d of c's receive buffer: the device path's ncclSend / ncclRecv pairs, as copies.
        for (std::size_t d = 0; d < P; ++d) {
            const std::size_t send_frames =
                plan.PerFrame() ? P * plan.MaxFramesPerCompositor() : F;
            std::vector<int> send(send_frames * band_pixels, -1);
            for (std::size_t f = 0; f < F; ++f) {
                const std::size_t cf = plan.Compositor(batch_index, f);
                std::copy_n(band_ids[d].begin() + f * band_pixels, band_pixels,
                            send.begin() + SendPixels(plan, cf, plan.Slot(f), band_pixels));
            }
            std::copy_n(send.begin() + SendPixels(plan, c, 0, band_pixels), n * band_pixels,
                        recv[c].begin() + plan.RecvSlot(c, d) * n * band_pixels);
        }
    }
    return recv;
}

// ---------------------------------------------------------------------------------------------
// Worker threads: one per local device; a job runs on every worker, the caller waits and watches.
// The first failure -- a worker's exception, or no progress on any device for the comm timeout --
// sets the shared abort flag (every worker's wait then throws), releases the host barrier and calls
// the owner's abort hook once (ncclCommAbort: RCCL kernels waiting on a peer that will never send
// exit, so the streams drain); the workers then get the same time again to return. Workers that
// still do not return (stuck in a HIP call behind a hung GPU) leave the pool wedged: it is never
// destroyed (its threads are never joined) and the engine refuses further work.

struct FrameEngine::Pool {
    Pool(std::size_t n, CommCtl* ctl, double timeout_s) : m_n(n), m_ctl(ctl), m_timeout(timeout_s) {
        for (std::size_t i = 0; i < n; ++i) {
            m_threads.emplace_back([this, i] { Loop(i); });
        }
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> lk(m_mu);
            m_stop = true;
        }
        m_cv.notify_all();
        for (auto& t : m_threads) {
            t.join();
        }
    }
    void Run(const std::function<void(std::size_t)>& job, const std::function<void()>& on_abort) {
        using Clock = std::chrono::steady_clock;
        const auto timeout = std::chrono::duration<double>(m_timeout);
        std::unique_lock<std::mutex> lk(m_mu);
        m_job = &job;
        m_pending = m_n;
        m_error = nullptr;
        m_aborted = false;
        m_bar_count = 0;
        ++m_gen;
        m_cv.notify_all();
        unsigned long seen = m_ctl->progress.load(std::memory_order_relaxed);
        auto last = Clock::now(), aborted_at = last;
        bool aborting = false;
        while (m_pending != 0) {
            m_done.wait_for(lk, std::chrono::milliseconds(20));
            if (m_pending == 0) {
                break;
            }
            const auto now = Clock::now();
            const unsigned long p = m_ctl->progress.load(std::memory_order_relaxed);
            if (p != seen) {
                seen = p;
                last = now;
            }
            if (!aborting && (m_error || now - last > timeout)) {
                if (!m_error) {
                    m_error = std::make_exception_ptr(std::runtime_error(
                        "frame engine: no device made progress in " + std::to_string(timeout.count()) +
                        " s (SRT_COMM_TIMEOUT_S); the run was aborted"));
                }
                aborting = true;
                aborted_at = now;
                m_aborted = true;
                m_ctl->abort.store(true);
                m_bar_cv.notify_all();
                lk.unlock();
                on_abort();
                lk.lock();
                continue;
            }
            if (aborting && now - aborted_at > timeout) {
                m_wedged = true;  // workers still inside HIP calls: never joined (see above)
                break;
            }
        }
        m_job = m_wedged ? m_job : nullptr;
        if (m_error && !aborting) {
            // Every worker returned, one with an error: RCCL work of the others may still wait on it.
            m_aborted = true;
            m_ctl->abort.store(true);
            lk.unlock();
            on_abort();
            lk.lock();
        }
        if (m_error) {
            std::exception_ptr e = m_error;
            if (m_wedged) {
                try {
                    std::rethrow_exception(e);
                } catch (const std::exception& x) {
                    throw std::runtime_error(std::string(x.what()) +
                                             "; a device worker did not return after the abort (GPU unresponsive)");
                }
            }
            std::rethrow_exception(e);
        }
    }
    void Barrier() {
        std::unique_lock<std::mutex> lk(m_mu);
        if (m_aborted) {
            throw std::runtime_error("another device's worker failed");
        }
        const std::size_t gen = m_bar_gen;
        if (++m_bar_count == m_n) {
            m_bar_count = 0;
            ++m_bar_gen;
            m_bar_cv.notify_all();
            return;
        }
        m_bar_cv.wait(lk, [&] { return m_bar_gen != gen || m_aborted; });
        if (m_bar_gen == gen) {
            throw std::runtime_error("another device's worker failed");
        }
    }
    bool wedged() const { return m_wedged; }

private:
    void Loop(std::size_t i) {
        std::size_t seen = 0;
        for (;;) {
            const std::function<void(std::size_t)>* job = nullptr;
            {
                std::unique_lock<std::mutex> lk(m_mu);
                m_cv.wait(lk, [&] { return m_stop || m_gen != seen; });
                if (m_stop) {
                    return;
                }
                seen = m_gen;
                job = m_job;
            }
            try {
                (*job)(i);
            } catch (...) {
                std::lock_guard<std::mutex> lk(m_mu);
                if (!m_error) {
                    m_error = std::current_exception();
                }
                m_aborted = true;
                m_bar_cv.notify_all();
            }
            std::lock_guard<std::mutex> lk(m_mu);
            if (--m_pending == 0) {
                m_done.notify_all();
            }
        }
    }

    std::size_t m_n;
    CommCtl* m_ctl;
    double m_timeout;
    std::vector<std::thread> m_threads;
    std::mutex m_mu;
    std::condition_variable m_cv, m_done, m_bar_cv;
    const std::function<void(std::size_t)>* m_job = nullptr;
    std::size_t m_gen = 0, m_pending = 0, m_bar_count = 0, m_bar_gen = 0;
    bool m_stop = false, m_aborted = false, m_wedged = false;
    std::exception_ptr m_error;
};

// ---------------------------------------------------------------------------------------------

struct FrameEngine::Queue {
    std::unique_ptr<DeviceScene> scene;
    hipStream_t stream = nullptr;
    hipEvent_t traced = nullptr;     // the batch's trace done (queue stream)
    hipEvent_t exchanged = nullptr;  // the batch's exchange done (comm stream)
    hipEvent_t drained = nullptr;    // end-of-run marker (queue stream), polled with a deadline
    // Id buffers of band frames, m_band_id_bytes each (int32 ids, or packed ids: render.h PackedIds).
    unsigned char* send = nullptr;   // bands: ids for the other compositors
    unsigned char* recv = nullptr;   // bands: [P][frames composited here][buffer rows][W] ids
    float* rgba = nullptr;           // frames rendered / composited here per batch, H x W x 4 each
    std::size_t rgba_frames = 0;
    std::size_t last_batch = 0;
    bool used = false;
};

struct FrameEngine::Device {
    int device = 0;
    std::size_t band = 0;  // global band / rank index
    hipStream_t comm = nullptr;
    hipEvent_t comm_drained = nullptr;
    // Exchange timing of the current run (pairs of timing events around each batch's group on
    // `comm`), summarised when the run ends (FrameEngine::exchange_stats).
    std::vector<hipEvent_t> xev;
    std::vector<char> xpend;  // per event: [2 slot] = the pair holds a group not yet added
    std::size_t xn = 0;
    double x_ms = 0.0, x_bytes = 0.0;
    std::size_t x_groups = 0;
    std::vector<Queue> queues;
    float* full = nullptr;  // inputs x H x W x 2
    float* band_in = nullptr;  // per role (FrameEngine::Role): inputs x the role's rows x W x 2
    std::size_t row_begin = 0, rows = 0;  // the band MeasureStages traces (kShare: the sender role)
    std::vector<Role> roles;
};

FrameEngine::FrameEngine(const Scene& scene, const std::vector<int>& devices, std::size_t width,
                         std::size_t height, const EngineOptions& options)
    : m_opt(options), m_width(width), m_height(height), m_world(devices.size()) {
    if (devices.empty()) {
        throw std::runtime_error("FrameEngine: no devices");
    }
    if (m_opt.rccl_self && devices.size() != 1) {
        throw std::runtime_error("FrameEngine: the RCCL self-exchange is a one-device option");
    }
    Init(scene, devices);
    m_copy = m_exchange && m_world > 1 && GatherByCopies(devices);
    try {
        if (m_exchange && !m_copy) {
            m_comms = CommInitAll(devices);
            m_comms_made = true;
        }
        SettleSplit();
        AllocateQueues();
        m_pool = std::make_unique<Pool>(m_dev.size(), m_ctl.get(), CommTimeoutSeconds());
    } catch (...) {
        Release();
        throw;
    }
}

FrameEngine::FrameEngine(const Scene& scene, int device, int rank, int world, const void* unique_id,
                         std::size_t width, std::size_t height, const EngineOptions& options)
    : m_opt(options), m_width(width), m_height(height), m_world(world < 1 ? 1 : static_cast<std::size_t>(world)),
      m_rank0(rank < 0 ? 0 : static_cast<std::size_t>(rank)) {
    if (rank < 0 || rank >= world) {
        throw std::runtime_error("FrameEngine: rank " + std::to_string(rank) + " outside world " +
                                 std::to_string(world));
    }
    if (m_opt.rccl_self) {
        throw std::runtime_error("FrameEngine: the RCCL self-exchange is a one-process option");
    }
    Init(scene, std::vector<int>{device});
    try {
        if (m_exchange && !m_opt.simulate) {
            if (unique_id == nullptr) {
                throw std::runtime_error("FrameEngine: a multi-rank band split needs the RCCL unique id");
            }
            m_comms.push_back(CommInitRank(device, world, unique_id, rank));
            m_comms_made = true;
        }
        SettleSplit();
        AllocateQueues();
        m_pool = std::make_unique<Pool>(1, m_ctl.get(), CommTimeoutSeconds());
    } catch (...) {
        Release();
        throw;
    }
}

std::string FrameEngine::PoolSelfTest(std::size_t workers, std::size_t failing, int mode, double timeout_s,
                                      double* elapsed_s, int* abort_calls) {
    CommCtl ctl;
    int calls = 0;
    const auto start = std::chrono::steady_clock::now();
    std::string error;
    {
        Pool pool(workers, &ctl, timeout_s);
        const std::function<void(std::size_t)> job = [&](std::size_t i) {
            if (i == failing && mode == Injection::kFail) {
                throw std::runtime_error("injected failure of worker " + std::to_string(i));
            }
            // Everyone else -- and the stalled worker -- waits like a worker behind a peer that will
            // never send: only the abort releases it (bounded, so a broken pool fails the test).
            while (!ctl.abort.load()) {
                if (std::chrono::steady_clock::now() - start > std::chrono::duration<double>(20 * timeout_s)) {
                    throw std::runtime_error("worker " + std::to_string(i) + " was never released");
                }
                std::this_thread::sleep_for(std::chrono::milliseconds(1));
            }
            throw std::runtime_error("worker " + std::to_string(i) + " released by the abort");
        };
        try {
            pool.Run(job, [&calls] { ++calls; });
        } catch (const std::exception& e) {
            error = e.what();
        }
    }
    if (elapsed_s != nullptr) {
        *elapsed_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - start).count();
    }
    if (abort_calls != nullptr) {
        *abort_calls = calls;
    }
    return error;
}

void FrameEngine::UniqueId(void* out128) {
    ncclUniqueId id;
    NcclCheck(ncclGetUniqueId(&id), "ncclGetUniqueId");
    static_assert(sizeof(id) == 128, "ncclUniqueId is 128 bytes");
    std::memcpy(out128, &id, sizeof(id));
}

void FrameEngine::Init(const Scene& scene, const std::vector<int>& devices) {
    if (m_width == 0 || m_height == 0) {
        throw std::runtime_error("FrameEngine: frame dimensions must be non-zero");
    }
    if (m_opt.batch == 0 || m_opt.batch > 4096 || m_opt.queues == 0 || m_opt.queues > 16) {
        throw std::runtime_error("FrameEngine: batch must be 1..4096 frames and queues 1..16");
    }
    if (m_opt.variant < kTraceLds || m_opt.variant > kTraceBvh) {
        throw std::runtime_error("FrameEngine: unknown trace variant " + std::to_string(m_opt.variant));
    }
    if (m_opt.exchange < EngineOptions::kAllToAll || m_opt.exchange > EngineOptions::kShare ||
        (m_opt.split != EngineOptions::kBands && m_opt.split != EngineOptions::kFrames)) {
        throw std::runtime_error("FrameEngine: unknown exchange or split");
    }
    m_bands = m_opt.split == EngineOptions::kBands;
    if (m_opt.rccl_self && !m_bands) {
        throw std::runtime_error("FrameEngine: the RCCL self-exchange needs the bands split");
    }
    m_exchange = m_bands && (m_world > 1 || m_opt.rccl_self);
    if (m_opt.launch == 0) {
        const char* v = std::getenv("SRT_LAUNCH_FRAMES");
        const long l = v == nullptr || *v == '\0' ? 0 : std::strtol(v, nullptr, 10);
        m_opt.launch = l > 0 ? static_cast<std::size_t>(l) : m_exchange ? kDefaultBandLaunch : kMaxBatch;
    }
    m_opt.launch = std::min({m_opt.launch, m_opt.batch, static_cast<std::size_t>(kMaxTableFrames)});
    {  // measurement only: whole frames (P = 1, or split frames) with deferred shading
        const char* v = std::getenv("SRT_DEFER_SHADE");
        m_defer_shade = v != nullptr && std::strcmp(v, "1") == 0 && !m_exchange;
    }
    m_inject = Injection::FromEnv();
    m_ctl = std::make_unique<CommCtl>();
    if (m_opt.exchange == EngineOptions::kShare && m_exchange && m_world > 1) {
        if (!m_opt.interleaved) {
            throw std::runtime_error("FrameEngine: the share exchange needs interleaved rows");
        }
        m_share = m_opt.share == 0 ? ShareAuto(m_height, m_world) : m_opt.share;
        if (m_share > 64 || (m_share & (m_share - 1)) != 0) {
            throw std::runtime_error("FrameEngine: share must be a power of two, 1..64 tile rows per cycle");
        }
    } else if (m_opt.exchange == EngineOptions::kShare) {
        m_opt.exchange = EngineOptions::kRotatingGather;  // one device: nothing to share
    }
    if (m_opt.rotate) {
        if (m_opt.interleaved || (m_opt.exchange != EngineOptions::kAllToAll && m_world > 1)) {
            throw std::runtime_error("FrameEngine: rotated bands need contiguous rows and the all-to-all exchange");
        }
        m_rotate = m_exchange && m_world > 1;  // one device: its band is the frame, nothing to rotate
    }
    m_plan.bands = m_bands ? m_world : 1;
    m_plan.batch = m_opt.batch;
    m_plan.exchange = m_opt.exchange;
    m_plan.rotate = m_rotate;
    m_scene = std::make_unique<Scene>(scene);
    m_n = scene.triangle_count();
    {  // the exchange payload: packed ids with the cull variant (env SRT_EXCHANGE_IDS=32: int32)
        const char* v = std::getenv("SRT_EXCHANGE_IDS");
        const bool force32 = v != nullptr && std::strcmp(v, "32") == 0;
        m_id_planes = m_exchange && m_opt.variant == kTraceCull && !force32 ? IdPlanes(m_n) : -1;
    }
    for (std::size_t i = 0; i < devices.size(); ++i) {
        auto d = std::make_unique<Device>();
        d->device = devices[i];
        d->band = m_rank0 + i;
        m_dev.push_back(std::move(d));
    }
    // The two-device split of rotated bands: the option, else env SRT_ROTATE_OWN, else (RCCL between
    // distinct devices) derived from the link measured once the communicators exist (SplitFromLink),
    // else the 80 % default.
    if (m_rotate && m_world == 2) {
        if (m_opt.own_rows != 0) {
            m_split_source = kSplitOption;
        } else if (RotateOwnPercent() != 0) {
            m_opt.own_rows = RotateOwnRows(m_height);
            m_split_source = kSplitEnv;
        } else {
            m_split_source = kSplitDefault;
        }
    }
    Layout(m_opt.own_rows);
}

// The band split, the id buffers' size and every device's roles for two-device own rows `own_rows`
// (0: the default; EngineSplit).
void FrameEngine::Layout(std::size_t own_rows) {
    // kShare: the frame's tile rows in cycles of k + P - 1 "classes" (the compositor's k, then one
    // per sender); the ids buffers hold one class.
    m_split = EngineSplit(m_height, m_world, m_bands, m_opt.interleaved, m_rotate, m_share, own_rows);
    {
        const std::size_t rows = m_split.BufferRows();
        m_band_id_bytes = m_id_planes >= 0 ? PackedIdLayout(m_id_planes, rows, m_width).bytes : rows * m_width * sizeof(int);
    }
    for (auto& d : m_dev) {
        d->roles.clear();
        if (m_share != 0) {
            const std::size_t classes = m_split.bands;
            Role own;
            own.pattern = RowPattern(classes, m_share);
            own.rows = PatternBandRows(m_height, 0, own.pattern);
            d->roles.push_back(own);
            for (std::size_t j = m_share; j < classes; ++j) {  // sender roles, in class order
                Role r;
                r.row_begin = m_split.RowBegin(j);
                r.rows = m_split.RowCount(j);
                r.pattern = classes;
                d->roles.push_back(r);
            }
        } else if (m_rotate) {  // role j = band j (contiguous); inputs read from the full frames
            for (std::size_t j = 0; j < m_world; ++j) {
                Role r;
                r.row_begin = m_split.RowBegin(j);
                r.rows = m_split.RowCount(j);
                r.pattern = 1;
                d->roles.push_back(r);
            }
        } else {
            Role r;
            r.row_begin = m_split.RowBegin(m_bands ? d->band : 0);
            r.rows = m_split.RowCount(m_bands ? d->band : 0);
            r.pattern = m_split.Interleave();
            d->roles.push_back(r);
        }
        std::size_t at = 0;
        for (Role& r : d->roles) {
            r.input = at;
            at += r.rows;
        }
    }
    for (std::size_t local = 0; local < m_dev.size(); ++local) {
        const Role& measured = m_dev[local]->roles[SenderRole(local)];
        m_dev[local]->row_begin = measured.row_begin;
        m_dev[local]->rows = measured.rows;
    }
}

// A role whose ids device `local` sends (they fit one band buffer of BufferRows rows): kShare its first
// sender class, rotate the band it traces for the next device's frames -- (p + c) % P for c = p + 1,
// never the compositor's own band 2c % P, which over two devices is larger than the buffer --, else its
// band. MeasureStages and PrimeSimulation trace it into a send buffer (they traced band
// d.band, the 864-row own band of device 0 at P = 2, into 216-row slots).
std::size_t FrameEngine::SenderRole(std::size_t local) const {
    if (m_share != 0) {
        return 1;
    }
    if (m_rotate) {
        return RoleOf(local, (m_dev[local]->band + 1) % m_world);
    }
    return 0;
}

std::size_t FrameEngine::RoleOf(std::size_t local, std::size_t c) const {
    if (m_rotate) {
        return m_plan.BandOf(m_dev[local]->band, c);
    }
    if (m_share == 0) {
        return 0;
    }
    const std::size_t self = m_dev[local]->band;
    return self == c ? 0 : 1 + m_plan.RecvSlot(c, self);
}

void FrameEngine::AllocateQueues() {
    const std::size_t frame_floats4 = m_width * m_height * 4;
    for (auto& dp : m_dev) {
        Device& d = *dp;
        DeviceGuard guard(d.device);
        HipCheck(hipStreamCreateWithFlags(&d.comm, hipStreamNonBlocking), "hipStreamCreate(comm)");
        HipCheck(hipEventCreateWithFlags(&d.comm_drained, hipEventDisableTiming), "hipEventCreate(comm drained)");
        d.queues.resize(m_opt.queues);
        for (Queue& q : d.queues) {
            HipCheck(hipStreamCreateWithFlags(&q.stream, hipStreamNonBlocking), "hipStreamCreate(queue)");
            HipCheck(hipEventCreateWithFlags(&q.traced, hipEventDisableTiming), "hipEventCreate(traced)");
            HipCheck(hipEventCreateWithFlags(&q.exchanged, hipEventDisableTiming), "hipEventCreate(exchanged)");
            HipCheck(hipEventCreateWithFlags(&q.drained, hipEventDisableTiming), "hipEventCreate(drained)");
            q.scene = std::make_unique<DeviceScene>(*m_scene, d.device);
            // one queue: nothing overlaps a batch's bin launches, so the trace recomputes the records
            q.scene->SetRecordMode(m_opt.queues == 1 ? kRecordsRecompute : kRecordsAuto);
            q.scene->Prepare(m_width, m_height, q.stream);
            if (m_exchange) {
                const std::size_t send_frames =
                    m_plan.PerFrame() ? m_world * m_plan.MaxFramesPerCompositor() : m_plan.batch;
                q.send = DeviceAlloc<unsigned char>(send_frames * m_band_id_bytes, "hipMalloc(send ids)");
                q.recv = DeviceAlloc<unsigned char>(m_world * m_plan.MaxFramesPerCompositor() * m_band_id_bytes,
                                          "hipMalloc(receive ids)");
                q.rgba_frames = m_plan.MaxFramesPerCompositor();
            } else {
                q.rgba_frames = m_opt.batch;
                if (m_defer_shade) {  // measurement: whole frames traced to ids, shaded by a second launch
                    q.recv = DeviceAlloc<unsigned char>(m_opt.batch * m_width * m_height * sizeof(int),
                                                        "hipMalloc(frame ids)");
                }
            }
            q.rgba = DeviceAlloc<float>(q.rgba_frames * frame_floats4, "hipMalloc(frames)");
        }
    }
}

// Rank mode (fewer local devices than the job has): the element-wise maximum of `v` over every rank
// (one ncclAllReduce on this process's communicator, waits polled with a deadline); otherwise `v`.
std::vector<double> FrameEngine::MaxOverRanks(const std::vector<double>& v) {
    if (m_dev.size() >= m_world || m_comms.empty() || v.empty()) {
        return v;
    }
    Device& d = *m_dev[0];
    DeviceGuard guard(d.device);
    double* buf = DeviceAlloc<double>(v.size(), "hipMalloc(allreduce)");
    hipStream_t st = nullptr;
    hipEvent_t done = nullptr;
    std::vector<double> out(v.size());
    try {
        HipCheck(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate(allreduce)");
        HipCheck(hipEventCreateWithFlags(&done, hipEventDisableTiming), "hipEventCreate(allreduce)");
        HipCheck(hipMemcpyAsync(buf, v.data(), v.size() * sizeof(double), hipMemcpyHostToDevice, st),
                 "hipMemcpyAsync(allreduce)");
        NcclCheck(ncclAllReduce(buf, buf, v.size(), ncclDouble, ncclMax, static_cast<ncclComm_t>(m_comms[0]), st),
                  "ncclAllReduce(engine setup)", true);
        CommSettle(&m_comms[0], 1, "allreduce enqueue (engine setup)", m_ctl.get());
        HipCheck(hipEventRecord(done, st), "hipEventRecord(allreduce)");
        CommWaitEvent(done, &m_comms[0], 1, "allreduce (engine setup)", m_ctl.get());
        HipCheck(hipMemcpy(out.data(), buf, v.size() * sizeof(double), hipMemcpyDeviceToHost), "hipMemcpy(allreduce)");
    } catch (...) {
        (void)hipFree(buf);
        if (done != nullptr) (void)hipEventDestroy(done);
        if (st != nullptr) (void)hipStreamDestroy(st);
        throw;
    }
    (void)hipFree(buf);
    (void)hipEventDestroy(done);
    (void)hipStreamDestroy(st);
    return out;
}

// The link: every local device sends kLinkProbeBytes to the next device of the job and receives as
// much from the previous one (two devices: both directions of their link at once, as the exchange
// does; one device with the self-exchange: to itself), in one group; 2 untimed and kLinkProbeReps
// timed groups, HIP events on each device's probe stream. GB/s per direction of the slowest device,
// over every rank.
double FrameEngine::MeasureLink() {
    constexpr std::size_t kLinkProbeBytes = std::size_t{32} << 20;
    constexpr int kLinkProbeReps = 5;
    const std::size_t n = m_dev.size();
    std::vector<unsigned char*> sbuf(n, nullptr), rbuf(n, nullptr);
    std::vector<hipStream_t> st(n, nullptr);
    std::vector<hipEvent_t> ev(2 * n, nullptr);
    double worst_ms = 0.0;
    auto release = [&] {
        for (std::size_t i = 0; i < n; ++i) {
            (void)hipSetDevice(m_dev[i]->device);
            (void)hipFree(sbuf[i]);
            (void)hipFree(rbuf[i]);
            for (int k = 0; k < 2; ++k) {
                if (ev[2 * i + k] != nullptr) (void)hipEventDestroy(ev[2 * i + k]);
            }
            if (st[i] != nullptr) (void)hipStreamDestroy(st[i]);
        }
    };
    try {
        for (std::size_t i = 0; i < n; ++i) {
            DeviceGuard guard(m_dev[i]->device);
            sbuf[i] = DeviceAlloc<unsigned char>(kLinkProbeBytes, "hipMalloc(link probe)");
            rbuf[i] = DeviceAlloc<unsigned char>(kLinkProbeBytes, "hipMalloc(link probe)");
            HipCheck(hipMemset(sbuf[i], 0x5A, kLinkProbeBytes), "hipMemset(link probe)");
            HipCheck(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking), "hipStreamCreate(link probe)");
            HipCheck(hipEventCreate(&ev[2 * i]), "hipEventCreate(link probe)");
            HipCheck(hipEventCreate(&ev[2 * i + 1]), "hipEventCreate(link probe)");
        }
        const auto group = [&] {
            NcclCheck(ncclGroupStart(), "ncclGroupStart(link probe)");
            ncclResult_t first = ncclSuccess;
            for (std::size_t i = 0; i < n; ++i) {
                const std::size_t self = m_dev[i]->band;
                const int to = static_cast<int>((self + 1) % m_world), from = static_cast<int>((self + m_world - 1) % m_world);
                auto comm = static_cast<ncclComm_t>(m_comms[i]);
                const ncclResult_t a = ncclSend(sbuf[i], kLinkProbeBytes, ncclUint8, to, comm, st[i]);
                const ncclResult_t b = ncclRecv(rbuf[i], kLinkProbeBytes, ncclUint8, from, comm, st[i]);
                for (const ncclResult_t r : {a, b}) {
                    if (r != ncclSuccess && r != ncclInProgress && first == ncclSuccess) {
                        first = r;
                    }
                }
            }
            const ncclResult_t end = ncclGroupEnd();
            NcclCheck(first, "ncclSend / ncclRecv (link probe)");
            NcclCheck(end, "ncclGroupEnd (link probe)", true);
            CommSettle(m_comms.data(), m_comms.size(), "link probe enqueue", m_ctl.get());
        };
        for (int r = 0; r < 2; ++r) {
            group();
        }
        for (std::size_t i = 0; i < n; ++i) {
            DeviceGuard guard(m_dev[i]->device);
            HipCheck(hipEventRecord(ev[2 * i], st[i]), "hipEventRecord(link probe)");
        }
        for (int r = 0; r < kLinkProbeReps; ++r) {
            group();
        }
        for (std::size_t i = 0; i < n; ++i) {
            DeviceGuard guard(m_dev[i]->device);
            HipCheck(hipEventRecord(ev[2 * i + 1], st[i]), "hipEventRecord(link probe)");
        }
        for (std::size_t i = 0; i < n; ++i) {
            DeviceGuard guard(m_dev[i]->device);
            CommWaitEvent(ev[2 * i + 1], m_comms.data(), m_comms.size(), "link probe", m_ctl.get());
            float ms = 0.f;
            HipCheck(hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]), "hipEventElapsedTime(link probe)");
            worst_ms = std::max(worst_ms, static_cast<double>(ms) / kLinkProbeReps);
        }
    } catch (...) {
        release();
        throw;
    }
    release();
    worst_ms = MaxOverRanks({worst_ms})[0];
    return worst_ms > 0.0 ? static_cast<double>(kLinkProbeBytes) / (worst_ms * 1e-3) / 1e9 : 0.0;
}

// One GPU's time per whole frame of this scene and resolution: 8-frame traces (uniform 0.5 offsets,
// RGBA, the N = 1 launch shape) on a scratch scene of each local device, one untimed and 3 timed
// launches; microseconds per frame of the slowest device, over every rank.
double FrameEngine::MeasureFrameUs() {
    constexpr std::size_t kFrames = kMaxBatch;
    constexpr int kReps = 3;
    double worst = 0.0;
    for (auto& dp : m_dev) {
        DeviceGuard guard(dp->device);
        DeviceScene s(*m_scene, dp->device);
        hipStream_t st = nullptr;
        hipEvent_t e0 = nullptr, e1 = nullptr;
        float* off = nullptr;
        float* rgba = nullptr;
        try {
            HipCheck(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate(frame probe)");
            HipCheck(hipEventCreate(&e0), "hipEventCreate(frame probe)");
            HipCheck(hipEventCreate(&e1), "hipEventCreate(frame probe)");
            off = DeviceAlloc<float>(FrameFloats(), "hipMalloc(frame probe offsets)");
            rgba = DeviceAlloc<float>(kFrames * m_width * m_height * 4, "hipMalloc(frame probe frames)");
            HipCheck(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(off), 0x3F000000, FrameFloats(), st),
                     "hipMemsetD32Async(frame probe offsets)");  // 0.5f
            s.Prepare(m_width, m_height, st);
            std::vector<const float*> offs(kFrames, off);
            std::vector<float*> outs(kFrames);
            for (std::size_t j = 0; j < kFrames; ++j) {
                outs[j] = rgba + j * m_width * m_height * 4;
            }
            const int variant = m_opt.variant;
            s.TraceBatch(offs.data(), outs.data(), nullptr, kFrames, 0, m_height, variant, st, 1);
            HipCheck(hipEventRecord(e0, st), "hipEventRecord(frame probe)");
            for (int r = 0; r < kReps; ++r) {
                s.TraceBatch(offs.data(), outs.data(), nullptr, kFrames, 0, m_height, variant, st, 1);
            }
            HipCheck(hipEventRecord(e1, st), "hipEventRecord(frame probe)");
            CommWaitEvent(e1, nullptr, 0, "frame probe", m_ctl.get());
            float ms = 0.f;
            HipCheck(hipEventElapsedTime(&ms, e0, e1), "hipEventElapsedTime(frame probe)");
            worst = std::max(worst, static_cast<double>(ms) * 1e3 / (kReps * kFrames));
        } catch (...) {
            (void)hipStreamSynchronize(st);
            (void)hipFree(off);
            (void)hipFree(rgba);
            if (e0 != nullptr) (void)hipEventDestroy(e0);
            if (e1 != nullptr) (void)hipEventDestroy(e1);
            if (st != nullptr) (void)hipStreamDestroy(st);
            throw;
        }
        (void)hipFree(off);
        (void)hipFree(rgba);
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        (void)hipStreamDestroy(st);
    }
    return MaxOverRanks({worst})[0];
}

// Once the communicators exist (RCCL engines only): the link rate (reported; srtEngineSplit), the
// two-device split derived from it when neither the option nor SRT_ROTATE_OWN chose one, and -- one
// rank per process -- a check that every rank uses the same split (ranks reading different
// environments would post mismatched send / receive sizes).
void FrameEngine::SettleSplit() {
    if (!m_comms_made) {
        return;
    }
    m_link_gbs = MeasureLink();
    if (m_rotate && m_world == 2 && m_split_source == kSplitDefault) {
        m_frame_us = MeasureFrameUs();
        const double bpp = static_cast<double>(m_band_id_bytes) / static_cast<double>(m_split.BufferRows() * m_width);
        m_opt.own_rows = RotateSplitForLink(m_height, m_width, m_link_gbs, m_frame_us, bpp);
        m_split_source = kSplitLink;
        Layout(m_opt.own_rows);
    }
    if (m_rotate && m_world == 2) {
        const double own = static_cast<double>(m_split.first_rows);
        const std::vector<double> r = MaxOverRanks({own, -own});
        if (r[0] != -r[1]) {
            throw std::runtime_error("FrameEngine: the ranks chose different two-device splits (own band rows " +
                                     std::to_string(static_cast<long>(-r[1])) + " .. " +
                                     std::to_string(static_cast<long>(r[0])) +
                                     "): set SRT_ROTATE_OWN alike on every rank, or leave it unset");
        }
    }
}

FrameEngine::SplitInfo FrameEngine::split_info() const {
    SplitInfo s;
    s.own_rows = m_rotate && m_world == 2 ? m_split.first_rows : 0;
    s.buffer_rows = m_split.BufferRows();
    s.link_gbs = m_link_gbs;
    s.frame_us = m_frame_us;
    s.source = m_split_source;
    return s;
}

FrameEngine::~FrameEngine() { Release(); }

void FrameEngine::AbortComms() noexcept {
    m_ctl->abort.store(true);
    std::unique_lock<std::shared_mutex> lk(m_ctl->mu);
    CommAbortAll(m_comms);
}

void FrameEngine::Release() noexcept {
    if (m_pool && m_pool->wedged()) {
        (void)m_pool.release();  // its threads are stuck in HIP calls: never joined (Pool above)
        m_wedged = true;
    }
    m_pool.reset();
    if (!m_failed.empty() && !m_comms.empty()) {
        AbortComms();  // a failed run: peers may never send what our RCCL kernels wait for
    }
    // Bounded drains: a wedged GPU must not turn the release into a hang.
    const double t = CommTimeoutSeconds();
    bool drained = !m_wedged;
    for (auto& dp : m_dev) {
        if (!dp || !drained) {
            continue;
        }
        (void)hipSetDevice(dp->device);
        for (Queue& q : dp->queues) {
            if (q.stream != nullptr && !StreamDrain(q.stream, t)) {
                drained = false;
            }
        }
        if (dp->comm != nullptr && drained && !StreamDrain(dp->comm, t)) {
            drained = false;
        }
    }
    if (!m_comms.empty()) {
        if (drained) {
            CommDestroyAll(m_comms);
        } else {
            AbortComms();
        }
    }
    if (!drained) {
        // Device memory still in use by work that never finished: hipFree would wait for it. Leak it.
        for (auto& dp : m_dev) {
            if (dp) {
                for (Queue& q : dp->queues) {
                    (void)q.scene.release();
                }
                (void)dp.release();
            }
        }
        m_dev.clear();
        return;
    }
    for (auto& dp : m_dev) {
        if (!dp) {
            continue;
        }
        (void)hipSetDevice(dp->device);
        for (Queue& q : dp->queues) {
            q.scene.reset();
            (void)hipFree(q.send);
            (void)hipFree(q.recv);
            (void)hipFree(q.rgba);
            q.send = q.recv = nullptr;
            q.rgba = nullptr;
            for (hipEvent_t* e : {&q.traced, &q.exchanged, &q.drained}) {
                if (*e != nullptr) {
                    (void)hipEventDestroy(*e);
                    *e = nullptr;
                }
            }
            if (q.stream != nullptr) {
                (void)hipStreamDestroy(q.stream);
            }
            q.stream = nullptr;
        }
        dp->queues.clear();
        (void)hipFree(dp->full);
        (void)hipFree(dp->band_in);
        dp->full = dp->band_in = nullptr;
        if (dp->comm_drained != nullptr) {
            (void)hipEventDestroy(dp->comm_drained);
            dp->comm_drained = nullptr;
        }
        for (hipEvent_t e : dp->xev) {
            (void)hipEventDestroy(e);
        }
        dp->xev.clear();
        dp->xpend.clear();
        if (dp->comm != nullptr) {
            (void)hipStreamDestroy(dp->comm);
            dp->comm = nullptr;
        }
    }
    m_dev.clear();
}

std::size_t FrameEngine::band_rows(std::size_t local) const { return local < m_dev.size() ? m_dev[local]->rows : 0; }

std::size_t FrameEngine::frames_rendered() const {
    return m_run_batches * m_opt.batch * (m_bands ? 1 : m_world);
}

double FrameEngine::exchange_bytes_per_frame() const {
    if (!m_exchange || m_world == 1) {
        return 0.0;
    }
    return static_cast<double>(m_world - 1) * static_cast<double>(m_band_id_bytes);
}

int* FrameEngine::Ids(unsigned char* buf, std::size_t band_frame) const {
    return reinterpret_cast<int*>(buf + band_frame * m_band_id_bytes);
}

std::size_t FrameEngine::FrameIndex(std::size_t local, std::size_t b, std::size_t f) const {
    // Split frames: each device renders frames of its own, device d's batch b being frames
    // (b * world + d) * F + f of the sequence; otherwise every device works on frames b * F + f.
    const std::size_t F = m_opt.batch;
    return m_bands ? b * F + f : (b * m_world + m_dev[local]->band) * F + f;
}

void FrameEngine::SetInputs(const float* host_offsets, std::size_t count) {
    if (host_offsets == nullptr || count == 0) {
        throw std::runtime_error("SetInputs: no input frames");
    }
    CheckUsable();
    if (m_exchange && count > 1 &&
        (count % m_opt.batch != 0 || (m_plan.PerFrame() && m_opt.batch % m_world != 0))) {
        throw std::runtime_error("SetInputs: with bands over " + std::to_string(m_world) + " devices, " +
                                 std::to_string(count) + " inputs need a multiple of the batch (" +
                                 std::to_string(m_opt.batch) + ") and a batch divisible by the devices");
    }
    if (m_defer_shade && count > 1 && count % m_opt.batch != 0) {
        // the deferred shading of a batch reads its inputs as one evenly strided run
        throw std::runtime_error("SetInputs: with SRT_DEFER_SHADE, " + std::to_string(count) +
                                 " inputs need a multiple of the batch (" + std::to_string(m_opt.batch) + ")");
    }
    const std::size_t ff = FrameFloats();
    for (auto& dp : m_dev) {
        Device& d = *dp;
        DeviceGuard guard(d.device);
        for (Queue& q : d.queues) {
            HipCheck(hipStreamSynchronize(q.stream), "hipStreamSynchronize(inputs)");
            q.used = false;  // frames of the previous inputs are no longer verifiable / readable
        }
        (void)hipFree(d.full);
        (void)hipFree(d.band_in);
        d.full = d.band_in = nullptr;
        d.full = DeviceAlloc<float>(count * ff, "hipMalloc(inputs)");
        HipCheck(hipMemcpy(d.full, host_offsets, count * ff * sizeof(float), hipMemcpyHostToDevice),
                 "hipMemcpy(inputs)");
        if (m_exchange && !m_rotate) {  // each role's rows of every input, band-local and contiguous
            const std::size_t row_floats = m_width * 2;
            std::size_t all_rows = 0;
            for (const Role& role : d.roles) {
                all_rows += role.rows;
            }
            std::vector<float> band(count * all_rows * row_floats);
            for (const Role& role : d.roles) {
                for (std::size_t r = 0; r < count; ++r) {
                    for (std::size_t y = 0; y < role.rows; ++y) {
                        const std::size_t fy = BandFrameRow(role.row_begin, role.pattern, y);
                        std::memcpy(band.data() + ((role.input * count) + r * role.rows + y) * row_floats,
                                    host_offsets + r * ff + fy * row_floats, row_floats * sizeof(float));
                    }
                }
            }
            d.band_in = DeviceAlloc<float>(band.size(), "hipMalloc(band inputs)");
            HipCheck(hipMemcpy(d.band_in, band.data(), band.size() * sizeof(float), hipMemcpyHostToDevice),
                     "hipMemcpy(band inputs)");
        }
    }
    m_inputs = count;
    if (m_opt.simulate && m_exchange) {
        PrimeSimulation();
    }
}

// Measurement (simulate: no peers, the exchange skipped): the compositor's deferred shading would
// read receive buffers nobody fills -- whatever the allocation held, hit statistics unlike a frame's.
// Fill them once, outside any run, with ids of this device's sender band (its trace of the first
// input: the hit density, regular tiles and packed layout of a real band), so the simulated shading
// does a real frame's work.
void FrameEngine::PrimeSimulation() {
    for (auto& dp : m_dev) {
        Device& d = *dp;
        DeviceGuard guard(d.device);
        const std::size_t local = static_cast<std::size_t>(&dp - &m_dev[0]);
        const std::size_t ri = SenderRole(local);
        const Role& role = d.roles[ri];
        for (Queue& q : d.queues) {
            if (q.send == nullptr || q.recv == nullptr || role.rows == 0) {
                continue;
            }
            const float* off = BandInput(local, 0, ri);
            int* ids = Ids(q.send, 0);
            q.scene->TraceBatch(&off, nullptr, &ids, 1, role.row_begin, role.rows, m_opt.variant, q.stream, role.pattern,
                                m_id_planes);
            const std::size_t slots = m_world * m_plan.MaxFramesPerCompositor();
            for (std::size_t k = 0; k < slots; ++k) {
                HipCheck(hipMemcpyAsync(q.recv + k * m_band_id_bytes, q.send, m_band_id_bytes, hipMemcpyDeviceToDevice,
                                        q.stream),
                         "hipMemcpyAsync(prime receive)");
            }
            HipCheck(hipStreamSynchronize(q.stream), "hipStreamSynchronize(prime)");
        }
    }
}

const float* FrameEngine::FullInput(std::size_t local, std::size_t k) const {
    return m_dev[local]->full + (k % m_inputs) * FrameFloats();
}

const float* FrameEngine::BandInput(std::size_t local, std::size_t k, std::size_t role) const {
    const Device& d = *m_dev[local];
    const Role& r = d.roles[role];
    if (m_rotate) {  // a contiguous band: its rows of the full input
        return FullInput(local, k) + r.row_begin * m_width * 2;
    }
    return d.band_in + (r.input * m_inputs + (k % m_inputs) * r.rows) * m_width * 2;
}

void FrameEngine::TracePhase(std::size_t local, std::size_t b) {
    Device& d = *m_dev[local];
    const std::size_t qi = b % m_opt.queues;
    Queue& q = d.queues[qi];
    const std::size_t F = m_opt.batch, k0 = b * F;
    if (m_exchange && q.used && !m_opt.simulate) {
        // This queue's send / receive buffers are free once its previous batch's exchange is done
        // (RCCL: on this device's comm stream; copies: every peer read our send buffer on its own).
        HipCheck(hipStreamWaitEvent(q.stream, q.exchanged, 0), "hipStreamWaitEvent(exchanged)");
        if (m_copy) {
            for (std::size_t p = 0; p < m_dev.size(); ++p) {
                if (p != local) {
                    HipCheck(hipStreamWaitEvent(q.stream, m_dev[p]->queues[qi].exchanged, 0),
                             "hipStreamWaitEvent(peer exchanged)");
                }
            }
        }
    }
    q.used = true;
    q.last_batch = b;
    const std::size_t L = m_opt.launch;
    std::vector<const float*> offs(L);
    std::vector<float*> rgba(L);
    std::vector<int*> ids(L);
    const std::size_t frame_floats4 = m_width * m_height * 4;
    if (!m_exchange) {  // whole frames, traced and shaded in one kernel
        const std::size_t frame_pixels = m_width * m_height;
        for (std::size_t f0 = 0; f0 < F; f0 += L) {
            const std::size_t n = std::min(L, F - f0);
            for (std::size_t j = 0; j < n; ++j) {
                offs[j] = FullInput(local, FrameIndex(local, b, f0 + j));
                rgba[j] = q.rgba + (f0 + j) * frame_floats4;
                ids[j] = m_defer_shade ? reinterpret_cast<int*>(q.recv) + (f0 + j) * frame_pixels : nullptr;
            }
            q.scene->TraceBatch(offs.data(), m_defer_shade ? nullptr : rgba.data(), m_defer_shade ? ids.data() : nullptr,
                                n, 0, m_height, m_opt.variant, q.stream, 1);
        }
        if (m_defer_shade) {  // inputs of one batch are evenly strided (SetInputs' condition)
            const std::size_t stride = m_inputs == 1 ? 0 : FrameFloats();
            q.scene->Shade(FullInput(local, FrameIndex(local, b, 0)), reinterpret_cast<const int*>(q.recv), q.rgba, 0,
                           m_height, q.stream, F,
                           m_height, 0, stride);
        }
        return;
    }
    const std::size_t self = d.band;
    if (m_share != 0) {
        TraceShare(local, b);
        HipCheck(hipEventRecord(q.traced, q.stream), "hipEventRecord(traced)");
        return;
    }
    if (m_rotate) {
        TraceRotated(local, b);
        HipCheck(hipEventRecord(q.traced, q.stream), "hipEventRecord(traced)");
        return;
    }
    const std::size_t ri = 0;
    const Role& role = d.roles[ri];
    if (role.rows != 0) {
        for (std::size_t f0 = 0; f0 < F; f0 += L) {
            const std::size_t n = std::min(L, F - f0);
            for (std::size_t j = 0; j < n; ++j) {
                const std::size_t f = f0 + j;
                const std::size_t c = m_plan.Compositor(b, f), slot = m_plan.Slot(f);
                offs[j] = BandInput(local, k0 + f, ri);
                // The compositor's own band is traced and shaded in one kernel straight into its frame
                // (RGBA at the band's frame rows; the deferred shading then skips that band), unless
                // the self-exchange option sends it through RCCL like every other band.
                const bool own = c == self && !m_opt.rccl_self;
                ids[j] = own ? nullptr : Ids(q.send, SendFrames(m_plan, c, slot));
                rgba[j] = own ? q.rgba + slot * frame_floats4 : nullptr;
            }
            q.scene->TraceBatch(offs.data(), rgba.data(), ids.data(), n, role.row_begin, role.rows, m_opt.variant,
                                q.stream, role.pattern, m_id_planes, true);
        }
    }
    HipCheck(hipEventRecord(q.traced, q.stream), "hipEventRecord(traced)");
}

// kShare: frame f's compositor c = f % P traces its own class rows (role 0) straight into the frame
// as RGBA; every other device traces its one class of f (role 1 + RecvSlot(c, self)) as packed ids
// into c's region of the send buffer. The sender classes of a batch differ only in their first row,
// so they share launches (per-frame row_begin), grouped by their row count (classes at the end of
// the frame may hold one tile row fewer).
void FrameEngine::TraceShare(std::size_t local, std::size_t b) {
    Device& d = *m_dev[local];
    Queue& q = d.queues[b % m_opt.queues];
    const std::size_t F = m_opt.batch, k0 = b * F, L = m_opt.launch, self = d.band;
    const std::size_t frame_floats4 = m_width * m_height * 4;
    std::vector<const float*> offs;
    std::vector<float*> rgba;
    std::vector<int*> ids;
    std::vector<std::size_t> begins;
    // The senders' tile rows are a small band of many frames: their launch sets take up to
    // SRT_SHARE_THIN_LAUNCH frames (default 256, the table's limit) to keep the launches few.
    static const std::size_t thin_launch = [] {
        const char* e = std::getenv("SRT_SHARE_THIN_LAUNCH");
        const long v = e != nullptr ? std::strtol(e, nullptr, 10) : 0;
        return v > 0 ? std::min<std::size_t>(static_cast<std::size_t>(v), kMaxTableFrames) : std::size_t{kMaxTableFrames};
    }();
    // The frames composited here are nearly whole frames: launch sets of SRT_SHARE_OWN_LAUNCH frames
    // (default 8, their parameters in the kernel arguments, as whole frames at P = 1; rank simulation
    // P = 2 / 4: 9.97 / 5.73 us per frame against 10.13 / 5.88 at 64, profiles/r04/share/ol_*).
    static const std::size_t own_launch = [] {
        const char* e = std::getenv("SRT_SHARE_OWN_LAUNCH");
        const long v = e != nullptr ? std::strtol(e, nullptr, 10) : 0;
        return v > 0 ? std::min<std::size_t>(static_cast<std::size_t>(v), kMaxTableFrames)
                     : static_cast<std::size_t>(kMaxBatch);
    }();
    const auto flush = [&](const Role& role, bool own) {
        const std::size_t LL = own ? own_launch : std::max(L, thin_launch);
        for (std::size_t f0 = 0; f0 < offs.size(); f0 += LL) {
            const std::size_t n = std::min(LL, offs.size() - f0);
            q.scene->TraceBatch(offs.data() + f0, own ? rgba.data() + f0 : nullptr, own ? nullptr : ids.data() + f0, n,
                                role.row_begin, role.rows, m_opt.variant, q.stream, role.pattern, m_id_planes, true,
                                own ? nullptr : begins.data() + f0);
        }
        offs.clear();
        rgba.clear();
        ids.clear();
        begins.clear();
    };
    // role 0: the frames composited here
    const Role& mine = d.roles[0];
    for (std::size_t f = self; f < F && mine.rows != 0; f += m_world) {
        offs.push_back(BandInput(local, k0 + f, 0));
        rgba.push_back(q.rgba + m_plan.Slot(f) * frame_floats4);
    }
    flush(mine, true);
    // the sender classes, by row count
    std::vector<std::size_t> counts;
    for (std::size_t ri = 1; ri < d.roles.size(); ++ri) {
        if (d.roles[ri].rows != 0 && std::find(counts.begin(), counts.end(), d.roles[ri].rows) == counts.end()) {
            counts.push_back(d.roles[ri].rows);
        }
    }
    for (const std::size_t rows : counts) {
        const Role* shape = nullptr;
        for (std::size_t f = 0; f < F; ++f) {
            const std::size_t c = m_plan.Compositor(b, f);
            if (c == self) {
                continue;
            }
            const std::size_t ri = RoleOf(local, c);
            const Role& role = d.roles[ri];
            if (role.rows != rows) {
                continue;
            }
            shape = &role;
            offs.push_back(BandInput(local, k0 + f, ri));
            ids.push_back(Ids(q.send, SendFrames(m_plan, c, m_plan.Slot(f))));
            begins.push_back(role.row_begin);
        }
        if (shape != nullptr) {
            flush(*shape, false);
        }
    }
}

// Rotated all-to-all: device `self` traces band BandOf(self, c) of a frame composited on device c --
// its own frames' band straight into the frame as RGBA, the others' as ids into c's region of the
// send buffer. Frames whose bands have the same row count share launches (per-frame first rows).
void FrameEngine::TraceRotated(std::size_t local, std::size_t b) {
    Device& d = *m_dev[local];
    Queue& q = d.queues[b % m_opt.queues];
    const std::size_t F = m_opt.batch, k0 = b * F, L = m_opt.launch, self = d.band;
    const std::size_t frame_floats4 = m_width * m_height * 4;
    std::vector<const float*> offs;
    std::vector<float*> rgba;
    std::vector<int*> ids;
    std::vector<std::size_t> begins;
    std::vector<std::size_t> counts;
    for (const Role& r : d.roles) {
        if (r.rows != 0 && std::find(counts.begin(), counts.end(), r.rows) == counts.end()) {
            counts.push_back(r.rows);
        }
    }
    for (const std::size_t rows : counts) {
        for (std::size_t f = 0; f < F; ++f) {
            const std::size_t c = m_plan.Compositor(b, f);
            const std::size_t j = RoleOf(local, c);
            const Role& role = d.roles[j];
            if (role.rows != rows) {
                continue;
            }
            const bool own = c == self;
            offs.push_back(BandInput(local, k0 + f, j));
            rgba.push_back(own ? q.rgba + m_plan.Slot(f) * frame_floats4 : nullptr);
            ids.push_back(own ? nullptr : Ids(q.send, SendFrames(m_plan, c, m_plan.Slot(f))));
            begins.push_back(role.row_begin);
        }
        for (std::size_t f0 = 0; f0 < offs.size(); f0 += L) {
            const std::size_t n = std::min(L, offs.size() - f0);
            q.scene->TraceBatch(offs.data() + f0, rgba.data() + f0, ids.data() + f0, n, begins[f0], rows, m_opt.variant,
                                q.stream, 1, m_id_planes, true, begins.data() + f0);
        }
        offs.clear();
        rgba.clear();
        ids.clear();
        begins.clear();
    }
}

// The next pair of timing events of device `local`'s exchange timing: a ring of 2 Q + 2 pairs (grown
// on demand up to that), a pair still holding an earlier group's times first waited for (polled with
// the comm deadline) and added to the run's total -- a bounded number of events however long the run
// (one new pair per batch, kept until Release).
hipEvent_t* FrameEngine::ExchangeEvents(std::size_t local) {
    Device& d = *m_dev[local];
    const std::size_t ring = 2 * m_opt.queues + 2, slot = d.xn % ring;
    while (d.xev.size() < 2 * (slot + 1)) {
        hipEvent_t e = nullptr;
        HipCheck(hipEventCreate(&e), "hipEventCreate(exchange timing)");
        d.xev.push_back(e);
        d.xpend.push_back(0);
    }
    if (d.xpend[2 * slot]) {
        AddExchangeTime(local, slot);
    }
    d.xpend[2 * slot] = 1;
    ++d.xn;
    return &d.xev[2 * slot];
}

void FrameEngine::AddExchangeTime(std::size_t local, std::size_t slot) {
    Device& d = *m_dev[local];
    const std::size_t nc = m_comms.empty() ? 0 : 1;
    CommWaitEvent(d.xev[2 * slot + 1], nc != 0 ? &m_comms[local] : nullptr, nc, "exchange timing", m_ctl.get());
    float ms = 0.f;
    HipCheck(hipEventElapsedTime(&ms, d.xev[2 * slot], d.xev[2 * slot + 1]), "hipEventElapsedTime(exchange)");
    d.x_ms += static_cast<double>(ms);
    ++d.x_groups;
    d.xpend[2 * slot] = 0;
}

double FrameEngine::SentBytes(std::size_t local, std::size_t b) const {
    const std::size_t self = m_dev[local]->band;
    double bytes = 0.0;
    for (std::size_t p = 0; p < m_world; ++p) {
        if (p != self || m_opt.rccl_self) {
            bytes += static_cast<double>(m_plan.FramesFor(b, p)) * static_cast<double>(m_band_id_bytes);
        }
    }
    return bytes;
}

FrameEngine::ExchangeStats FrameEngine::exchange_stats(std::size_t local) const {
    ExchangeStats st;
    if (local < m_dev.size()) {
        const Device& d = *m_dev[local];
        st.groups = d.x_groups;
        st.ms_mean = d.x_groups != 0 ? d.x_ms / static_cast<double>(d.x_groups) : 0.0;
        st.bytes_sent = d.x_groups != 0 ? d.x_bytes / static_cast<double>(d.x_groups) : 0.0;
    }
    return st;
}

void FrameEngine::ExchangePhase(std::size_t local, std::size_t b) {
    Device& d = *m_dev[local];
    Queue& q = d.queues[b % m_opt.queues];
    const std::size_t self = d.band, n_self = m_plan.FramesFor(b, self);
    HipCheck(hipStreamWaitEvent(d.comm, q.traced, 0), "hipStreamWaitEvent(traced)");
    hipEvent_t* xe = ExchangeEvents(local);
    d.x_bytes += SentBytes(local, b);
    HipCheck(hipEventRecord(xe[0], d.comm), "hipEventRecord(exchange start)");
    {
        // The communicator is touched only under the shared lock and before an abort (comm.h).
        std::shared_lock<std::shared_mutex> lk(m_ctl->mu);
        if (m_ctl->abort.load()) {
            throw std::runtime_error("exchange: aborted (another device's worker failed)");
        }
        auto comm = static_cast<ncclComm_t>(m_comms[local]);
        NcclCheck(ncclGroupStart(), "ncclGroupStart");
        ncclResult_t first = ncclSuccess;
        auto note = [&first](ncclResult_t r) {
            if (r != ncclSuccess && r != ncclInProgress && first == ncclSuccess) {
                first = r;
            }
        };
        for (std::size_t p = 0; p < m_world; ++p) {
            if (p == self && !m_opt.rccl_self) {
                continue;
            }
            const std::size_t n_p = m_plan.FramesFor(b, p);
            if (n_p != 0) {
                note(ncclSend(q.send + SendFrames(m_plan, p, 0) * m_band_id_bytes, n_p * m_band_id_bytes, ncclUint8,
                              static_cast<int>(p), comm, d.comm));
            }
            if (n_self != 0) {
                note(ncclRecv(q.recv + m_plan.RecvSlot(self, p) * n_self * m_band_id_bytes, n_self * m_band_id_bytes,
                              ncclUint8,
                              static_cast<int>(p),
                              comm, d.comm));
            }
        }
        const ncclResult_t end = ncclGroupEnd();
        NcclCheck(first, "ncclSend / ncclRecv (band ids)");
        NcclCheck(end, "ncclGroupEnd (band ids)", true);
    }
    // Nonblocking communicator: the group's kernels are on the comm stream once it settles.
    CommSettle(&m_comms[local], 1, "exchange enqueue (band ids)", m_ctl.get());
    HipCheck(hipEventRecord(xe[1], d.comm), "hipEventRecord(exchange end)");
    HipCheck(hipEventRecord(q.exchanged, d.comm), "hipEventRecord(exchanged)");
}

void FrameEngine::CopyPhase(std::size_t local, std::size_t b) {
    Device& d = *m_dev[local];
    const std::size_t qi = b % m_opt.queues;
    Queue& q = d.queues[qi];
    const std::size_t self = d.band, n_self = m_plan.FramesFor(b, self);
    HipCheck(hipStreamWaitEvent(d.comm, q.traced, 0), "hipStreamWaitEvent(traced)");
    hipEvent_t* xe = ExchangeEvents(local);
    d.x_bytes += SentBytes(local, b);
    HipCheck(hipEventRecord(xe[0], d.comm), "hipEventRecord(exchange start)");
    if (n_self != 0) {
        for (std::size_t p = 0; p < m_dev.size(); ++p) {
            if (p == local) {
                continue;
            }
            Device& peer = *m_dev[p];
            Queue& pq = peer.queues[qi];
            HipCheck(hipStreamWaitEvent(d.comm, pq.traced, 0), "hipStreamWaitEvent(peer traced)");
            HipCheck(hipMemcpyPeerAsync(q.recv + m_plan.RecvSlot(self, peer.band) * n_self * m_band_id_bytes, d.device,
                                        pq.send + SendFrames(m_plan, self, 0) * m_band_id_bytes, peer.device,
                                        n_self * m_band_id_bytes, d.comm),
                     "hipMemcpyPeerAsync(band ids)");
        }
    }
    HipCheck(hipEventRecord(xe[1], d.comm), "hipEventRecord(exchange end)");
    HipCheck(hipEventRecord(q.exchanged, d.comm), "hipEventRecord(exchanged)");
}

void FrameEngine::ShadePhase(std::size_t local, std::size_t b) {
    Device& d = *m_dev[local];
    Queue& q = d.queues[b % m_opt.queues];
    const std::size_t self = d.band, n_self = m_plan.FramesFor(b, self);
    if (n_self == 0) {
        return;
    }
    if (!m_opt.simulate) {
        HipCheck(hipStreamWaitEvent(q.stream, q.exchanged, 0), "hipStreamWaitEvent(exchanged)");
    }
    // The compositor's frames in slot order read evenly strided inputs (SetInputs' condition).
    const std::size_t F = m_opt.batch, k0 = b * F;
    const bool a2a = m_plan.PerFrame();
    const std::size_t first = k0 + (a2a ? self : 0);
    const std::size_t stride = m_inputs == 1 ? 0 : (a2a ? m_world : 1) * FrameFloats();
    // The compositor's own rows are RGBA already: its band (all-to-all, rotating), or the first
    // m_share classes (share; the received ids start at class m_share).
    const long skip = m_opt.rccl_self || m_share != 0 ? -1 : static_cast<long>(m_plan.BandOf(self, self));
    q.scene->Shade(FullInput(local, first), reinterpret_cast<const int*>(q.recv), q.rgba, 0, m_height, q.stream, n_self,
                   m_split.BufferRows(), m_split.interleaved ? m_split.bands : 0, stride, m_id_planes, skip, m_share,
                   m_split.interleaved ? 0 : m_split.first_rows);
}

void FrameEngine::Inject(std::size_t local, std::size_t b) {
    if (m_inject.kind == Injection::kNone || m_inject.local != local || m_inject.batch != b) {
        return;
    }
    const std::string where = "local device " + std::to_string(local) + ", batch " + std::to_string(b);
    if (m_inject.kind == Injection::kFail) {
        throw std::runtime_error("injected failure (SRT_ENGINE_INJECT) on " + where);
    }
    // A stall: this worker stops making progress, as one stuck behind a dead peer would, until the
    // run is aborted (bounded, so a broken watchdog shows as a test failure rather than a hang).
    const auto start = std::chrono::steady_clock::now();
    while (!m_ctl->abort.load()) {
        if (std::chrono::steady_clock::now() - start > std::chrono::duration<double>(10 * CommTimeoutSeconds())) {
            throw std::runtime_error("injected stall (SRT_ENGINE_INJECT) on " + where + " was never aborted");
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    throw std::runtime_error("injected stall (SRT_ENGINE_INJECT) on " + where + " ended by the abort");
}

void FrameEngine::RunWorker(std::size_t local, std::size_t b0, std::size_t batches) {
    Device& d = *m_dev[local];
    DeviceGuard guard(d.device);
    d.xn = 0;
    std::fill(d.xpend.begin(), d.xpend.end(), 0);  // a failed run's pairs: not this run's groups
    d.x_ms = d.x_bytes = 0.0;
    d.x_groups = 0;
    const std::size_t nc = m_comms.empty() ? 0 : 1;
    void* const* comm = nc != 0 ? &m_comms[local] : nullptr;
    for (std::size_t b = b0; b < b0 + batches; ++b) {
        Inject(local, b);
        if (m_ctl->abort.load(std::memory_order_relaxed)) {
            throw std::runtime_error("run aborted: another device's worker failed");
        }
        static const bool probe = std::getenv("SRT_PROBE_HOST") != nullptr;
        const auto tp0 = std::chrono::steady_clock::now();
        TracePhase(local, b);
        const auto tp1 = std::chrono::steady_clock::now();
        if (probe) {
            const double us = std::chrono::duration<double, std::micro>(tp1 - tp0).count();
            if (us > 300.0) {
                std::fprintf(stderr, "[probe] batch %zu trace phase %.0f us\n", b, us);
            }
        }
        if (m_exchange) {
            if (m_opt.simulate) {
                ShadePhase(local, b);  // no peers: the exchange is skipped (measurement)
                if (probe) {
                    const double us =
                        std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - tp1).count();
                    if (us > 300.0) {
                        std::fprintf(stderr, "[probe] batch %zu shade phase %.0f us\n", b, us);
                    }
                }
            } else if (m_copy) {
                Barrier();  // every device's trace of batch b is enqueued (its `traced` recorded)
                CopyPhase(local, b);
                Barrier();  // every `exchanged` recorded before any device reuses a send buffer
                ShadePhase(local, b);
            } else {
                ExchangePhase(local, b);
                ShadePhase(local, b);
            }
        }
        m_ctl->progress.fetch_add(1, std::memory_order_relaxed);
    }
    // The end of the run: every queue and the exchange stream drained, each wait bounded and
    // abortable (comm.h), never a bare hipStreamSynchronize behind RCCL.
    for (Queue& q : d.queues) {
        HipCheck(hipEventRecord(q.drained, q.stream), "hipEventRecord(drained)");
    }
    HipCheck(hipEventRecord(d.comm_drained, d.comm), "hipEventRecord(comm drained)");
    for (Queue& q : d.queues) {
        CommWaitEvent(q.drained, comm, nc, "render (queue)", m_ctl.get());
    }
    CommWaitEvent(d.comm_drained, comm, nc, "render (exchange)", m_ctl.get());
    for (std::size_t slot = 0; 2 * slot < d.xev.size(); ++slot) {  // the groups not added yet (drained above)
        if (d.xpend[2 * slot]) {
            AddExchangeTime(local, slot);
        }
    }
}

void FrameEngine::Barrier() {
    if (m_pool) {
        m_pool->Barrier();
    }
}

void FrameEngine::CheckUsable() const {
    if (!m_failed.empty()) {
        throw std::runtime_error("frame engine stopped after an earlier failure (" + m_failed +
                                 "); create a new engine");
    }
}

void FrameEngine::Run(std::size_t batches) {
    if (m_inputs == 0) {
        throw std::runtime_error("Run: SetInputs() has not been called");
    }
    CheckUsable();
    const std::size_t b0 = m_next_batch;
    m_run_batches = batches;
    if (batches == 0) {
        return;
    }
    m_next_batch += batches;
    // On the heap: a worker that never returns from a failed run (a wedged pool) is still inside this
    // closure, so it is then leaked with the pool rather than destroyed under it (srtEngineRelease
    // leaks a wedged engine too: the worker's `this`).
    auto job = std::make_unique<std::function<void(std::size_t)>>(
        [this, b0, batches](std::size_t i) { RunWorker(i, b0, batches); });
    try {
        m_pool->Run(*job, [this] { AbortComms(); });
    } catch (const std::exception& e) {
        if (m_pool->wedged()) {
            (void)job.release();
            m_wedged = true;
        }
        m_failed = e.what();
        if (!m_comms.empty()) {
            AbortComms();
        }
        throw;
    }
}

bool FrameEngine::ReadFrame(std::size_t k, float* host_rgba) {
    const std::size_t F = m_opt.batch;
    // Frame k's batch and device (FrameIndex inverted): split frames deal each batch's frames to
    // the devices F at a time.
    const std::size_t per_batch = m_bands ? F : F * m_world;
    const std::size_t b = k / per_batch, within = k % per_batch, f = within % F;
    if (b >= m_next_batch || b + m_opt.queues < m_next_batch) {
        return false;
    }
    std::size_t local = 0, slot = f;
    if (!m_bands) {
        const std::size_t dev = within / F;
        if (dev < m_rank0 || dev >= m_rank0 + m_dev.size()) {
            return false;
        }
        local = dev - m_rank0;
    } else if (m_exchange) {
        const std::size_t c = m_plan.Compositor(b, f);
        if (c < m_rank0 || c >= m_rank0 + m_dev.size()) {
            return false;
        }
        local = c - m_rank0;
        slot = m_plan.Slot(f);
    }
    Device& d = *m_dev[local];
    Queue& q = d.queues[b % m_opt.queues];
    if (!q.used || q.last_batch != b) {
        return false;
    }
    DeviceGuard guard(d.device);
    CheckUsable();
    HipCheck(hipStreamSynchronize(q.stream), "hipStreamSynchronize(read frame)");
    const std::size_t frame_floats4 = m_width * m_height * 4;
    HipCheck(hipMemcpy(host_rgba, q.rgba + slot * frame_floats4, frame_floats4 * sizeof(float), hipMemcpyDeviceToHost),
             "hipMemcpy(read frame)");
    return true;
}

std::size_t FrameEngine::Verify(std::size_t* checked, std::size_t per_queue) {
    const std::size_t F = m_opt.batch;
    const std::size_t frame_floats4 = m_width * m_height * 4;
    CheckUsable();
    std::size_t bad = 0, count = 0;
    std::vector<float> got(frame_floats4);
    for (std::size_t local = 0; local < m_dev.size(); ++local) {
        Device& d = *m_dev[local];
        DeviceGuard guard(d.device);
        // Reference: one full-frame fused trace per input on a fresh scene of this device.
        DeviceScene ref_scene(*m_scene, d.device);
        hipStream_t st = nullptr;
        HipCheck(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate(verify)");
        float* ref_dev = nullptr;
        std::vector<std::vector<float>> refs(m_inputs);
        try {
            ref_dev = DeviceAlloc<float>(frame_floats4, "hipMalloc(verify)");
            ref_scene.Prepare(m_width, m_height, st);
            for (Queue& q : d.queues) {
                if (!q.used) {
                    continue;
                }
                HipCheck(hipStreamSynchronize(q.stream), "hipStreamSynchronize(verify)");
                const std::size_t b = q.last_batch;
                std::size_t taken = 0;
                for (std::size_t f = 0; f < F && taken < per_queue; ++f) {
                    std::size_t slot = f;
                    if (m_exchange) {
                        if (m_plan.Compositor(b, f) != d.band) {
                            continue;
                        }
                        slot = m_plan.Slot(f);
                    }
                    ++taken;
                    const std::size_t r = FrameIndex(local, b, f) % m_inputs;
                    if (refs[r].empty()) {
                        ref_scene.Trace(FullInput(local, r), ref_dev, 0, m_height, m_opt.variant == kTraceCull ? kTraceLds
                                                                                                              : kTraceCull,
                                        st);
                        HipCheck(hipStreamSynchronize(st), "verify render");
                        refs[r].resize(frame_floats4);
                        HipCheck(hipMemcpy(refs[r].data(), ref_dev, frame_floats4 * sizeof(float),
                                           hipMemcpyDeviceToHost),
                                 "hipMemcpy(verify reference)");
                    }
                    HipCheck(hipMemcpy(got.data(), q.rgba + slot * frame_floats4, frame_floats4 * sizeof(float),
                                       hipMemcpyDeviceToHost),
                             "hipMemcpy(verify frame)");
                    ++count;
                    if (std::memcmp(got.data(), refs[r].data(), frame_floats4 * sizeof(float)) != 0) {
                        ++bad;
                    }
                }
            }
        } catch (...) {
            (void)hipFree(ref_dev);
            (void)hipStreamDestroy(st);
            throw;
        }
        (void)hipFree(ref_dev);
        (void)hipStreamDestroy(st);
    }
    if (checked != nullptr) {
        *checked = count;
    }
    return bad;
}

DeviceScene::StageTimes FrameEngine::MeasureStages(std::size_t local, std::size_t launches, std::size_t frames) {
    if (local >= m_dev.size()) {
        throw std::runtime_error("MeasureStages: no local device " + std::to_string(local));
    }
    CheckUsable();
    frames = std::max<std::size_t>(1, frames);
    if (frames > m_opt.batch || frames > static_cast<std::size_t>(kMaxTableFrames)) {
        throw std::runtime_error("MeasureStages: at most the batch (" + std::to_string(m_opt.batch) +
                                 ") frames per launch");
    }
    if (m_inputs == 0) {
        throw std::runtime_error("MeasureStages: SetInputs() has not been called");
    }
    Device& d = *m_dev[local];
    DeviceGuard guard(d.device);
    Queue& q = d.queues[0];
    for (Queue& qq : d.queues) {
        HipCheck(hipStreamSynchronize(qq.stream), "hipStreamSynchronize(stages)");
    }
    HipCheck(hipStreamSynchronize(d.comm), "hipStreamSynchronize(stages)");
    q.scene->TakeTimes();
    q.scene->SetTiming(true);
    const std::size_t frame_floats4 = m_width * m_height * 4;
    std::vector<const float*> offs(frames);
    std::vector<float*> rgba(frames);
    std::vector<int*> ids(frames);
    try {
        for (std::size_t i = 0; i < launches; ++i) {
            for (std::size_t j = 0; j < frames; ++j) {
                const std::size_t k = i * frames + j;
                offs[j] = m_exchange ? BandInput(local, k) : FullInput(local, k);
                rgba[j] = q.rgba + j * frame_floats4;
                ids[j] = Ids(q.send, j);
            }
            if (m_exchange) {
                // a sender role: its ids fit the send buffer's band frames (SenderRole)
                const std::size_t ri = SenderRole(local);
                const Role& role = d.roles[ri];
                for (std::size_t j = 0; j < frames; ++j) {
                    offs[j] = BandInput(local, i * frames + j, ri);
                }
                if (role.rows != 0) {
                    q.scene->TraceBatch(offs.data(), nullptr, ids.data(), frames, role.row_begin, role.rows, m_opt.variant,
                                        q.stream, role.pattern, m_id_planes);
                }
            } else {
                q.scene->TraceBatch(offs.data(), rgba.data(), nullptr, frames, 0, m_height, m_opt.variant, q.stream, 1);
            }
        }
    } catch (...) {
        q.scene->SetTiming(false);
        throw;
    }
    q.scene->SetTiming(false);
    const DeviceScene::StageTimes t = q.scene->TakeTimes();
    q.used = false;  // its buffers now hold measurement frames, not a batch (Verify / ReadFrame skip it)
    return t;
}

}  // namespace srt
