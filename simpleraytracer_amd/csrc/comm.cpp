#include "comm.h"

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <thread>

#include "renderer.h"

namespace srt {
namespace {

using Clock = std::chrono::steady_clock;

// Polling cadence: a yield-only spin for the first 200 us (the end of a timed run waits here), then
// 50-us sleeps so a long wait does not burn a host core.
class Poller {
public:
    explicit Poller(double timeout_s) : m_start(Clock::now()), m_timeout(timeout_s > 0 ? timeout_s : CommTimeoutSeconds()) {}
    void Pause() {
        if (Clock::now() - m_start < std::chrono::microseconds(200)) {
            std::this_thread::yield();
        } else {
            std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
    }
    bool Expired() const { return Seconds() > m_timeout; }
    double Seconds() const { return std::chrono::duration<double>(Clock::now() - m_start).count(); }
    double timeout() const { return m_timeout; }

private:
    Clock::time_point m_start;
    double m_timeout;
};

// The first communicator reporting an error (ncclSuccess when none, ncclInProgress when one is
// still busy and none failed).
ncclResult_t AsyncState(void* const* comms, std::size_t n) {
    ncclResult_t worst = ncclSuccess;
    for (std::size_t i = 0; i < n; ++i) {
        if (comms[i] == nullptr) {
            continue;
        }
        ncclResult_t st = ncclSuccess;
        const ncclResult_t r = ncclCommGetAsyncError(static_cast<ncclComm_t>(comms[i]), &st);
        if (r != ncclSuccess) {
            return r;
        }
        if (st != ncclSuccess && st != ncclInProgress) {
            return st;
        }
        if (st == ncclInProgress) {
            worst = ncclInProgress;
        }
    }
    return worst;
}

[[noreturn]] void Fail(const char* what, const std::string& why) {
    throw std::runtime_error(std::string("RCCL error: ") + what + ": " + why);
}

// AsyncState under the owner's shared lock, refusing once the owner has begun to abort (the
// communicators may be freed from then on).
ncclResult_t GuardedState(void* const* comms, std::size_t n, const char* what, CommCtl* ctl) {
    if (ctl == nullptr) {
        return AsyncState(comms, n);
    }
    std::shared_lock<std::shared_mutex> lk(ctl->mu);
    if (ctl->abort.load(std::memory_order_relaxed)) {
        Fail(what, "aborted: another device's worker failed");
    }
    return AsyncState(comms, n);
}

}  // namespace

double CommTimeoutSeconds() {
    const char* v = std::getenv("SRT_COMM_TIMEOUT_S");
    if (v != nullptr && *v != '\0') {
        const double s = std::strtod(v, nullptr);
        if (s > 0) {
            return s;
        }
    }
    return 60.0;
}

void NcclCheck(ncclResult_t res, const char* what, bool in_progress_ok) {
    if (res == ncclSuccess || (in_progress_ok && res == ncclInProgress)) {
        return;
    }
    Fail(what, ncclGetErrorString(res));
}

void CommSettle(void* const* comms, std::size_t n, const char* what, CommCtl* ctl, double timeout_s) {
    Poller poll(timeout_s);
    for (;;) {
        const ncclResult_t st = GuardedState(comms, n, what, ctl);
        if (st == ncclSuccess) {
            return;
        }
        if (st != ncclInProgress) {
            Fail(what, ncclGetErrorString(st));
        }
        if (poll.Expired()) {
            Fail(what, "no progress in " + std::to_string(poll.timeout()) +
                           " s (a peer stopped or never joined; SRT_COMM_TIMEOUT_S)");
        }
        poll.Pause();
    }
}

std::vector<void*> CommInitAll(const std::vector<int>& devices) {
    ncclUniqueId id;
    NcclCheck(ncclGetUniqueId(&id), "ncclGetUniqueId");
    std::vector<void*> comms(devices.size(), nullptr);
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    NcclCheck(ncclGroupStart(), "ncclGroupStart(init)");
    ncclResult_t first = ncclSuccess;
    for (std::size_t i = 0; i < devices.size(); ++i) {
        DeviceGuard guard(devices[i]);
        ncclComm_t c = nullptr;
        const ncclResult_t r = ncclCommInitRankConfig(&c, static_cast<int>(devices.size()), id, static_cast<int>(i), &cfg);
        comms[i] = c;
        if (r != ncclSuccess && r != ncclInProgress && first == ncclSuccess) {
            first = r;
        }
    }
    const ncclResult_t end = ncclGroupEnd();
    try {
        NcclCheck(first, "ncclCommInitRankConfig");
        NcclCheck(end, "ncclGroupEnd(init)", true);
        CommSettle(comms.data(), comms.size(), "communicator setup", nullptr, 2 * CommTimeoutSeconds());
    } catch (...) {
        CommAbortAll(comms);
        throw;
    }
    return comms;
}

void* CommInitRank(int device, int world, const void* unique_id128, int rank) {
    if (unique_id128 == nullptr) {
        throw std::runtime_error("RCCL error: a multi-rank communicator needs the unique id");
    }
    DeviceGuard guard(device);
    ncclUniqueId id;
    static_assert(sizeof(id) == 128, "ncclUniqueId is 128 bytes");
    std::memcpy(&id, unique_id128, sizeof(id));
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclComm_t c = nullptr;
    const ncclResult_t r = ncclCommInitRankConfig(&c, world, id, rank, &cfg);
    std::vector<void*> comms{c};
    try {
        NcclCheck(r, "ncclCommInitRankConfig", true);
        CommSettle(comms.data(), 1, "communicator setup", nullptr, 2 * CommTimeoutSeconds());
    } catch (...) {
        CommAbortAll(comms);
        throw;
    }
    return c;
}

void CommWaitEvent(hipEvent_t ev, void* const* comms, std::size_t n, const char* what, CommCtl* ctl,
                   double timeout_s) {
    Poller poll(timeout_s);
    for (unsigned i = 0;; ++i) {
        const hipError_t q = hipEventQuery(ev);
        if (q == hipSuccess) {
            if (ctl != nullptr) {
                ctl->progress.fetch_add(1, std::memory_order_relaxed);
            }
            return;
        }
        if (q != hipErrorNotReady) {
            HipCheck(q, what);
        }
        if ((i & 15u) == 0) {  // the async-error query takes RCCL's lock: every 16th poll
            const ncclResult_t st = GuardedState(comms, n, what, ctl);
            if (st != ncclSuccess && st != ncclInProgress) {
                Fail(what, ncclGetErrorString(st));
            }
        } else if (ctl != nullptr && ctl->abort.load(std::memory_order_relaxed)) {
            Fail(what, "aborted: another device's worker failed");
        }
        if (poll.Expired()) {
            Fail(what, "not complete after " + std::to_string(poll.timeout()) +
                           " s (a peer stopped progressing; SRT_COMM_TIMEOUT_S)");
        }
        poll.Pause();
    }
}

bool StreamDrain(hipStream_t stream, double timeout_s) noexcept {
    Poller poll(timeout_s);
    for (;;) {
        const hipError_t q = hipStreamQuery(stream);
        if (q == hipSuccess) {
            return true;
        }
        if (q != hipErrorNotReady || poll.Expired()) {
            return false;
        }
        poll.Pause();
    }
}

void CommAbortAll(std::vector<void*>& comms) noexcept {
    for (void* c : comms) {
        if (c != nullptr) {
            (void)ncclCommAbort(static_cast<ncclComm_t>(c));
        }
    }
    comms.clear();
}

void CommDestroyAll(std::vector<void*>& comms) noexcept {
    // Every finalize first, inside one group (the ranks of one ncclCommInitAll world may wait for
    // their peers' finalize: one at a time, each would wait out its settle limit), then one settle
    // for all of them, then the destroys. Anything that fails is aborted instead.
    std::vector<void*> live;
    for (void* c : comms) {
        if (c != nullptr) {
            live.push_back(c);
        }
    }
    comms.clear();
    if (live.empty()) {
        return;
    }
    bool ok = true;
    try {
        NcclCheck(ncclGroupStart(), "ncclGroupStart(finalize)");
        ncclResult_t first = ncclSuccess;
        for (void* c : live) {
            const ncclResult_t r = ncclCommFinalize(static_cast<ncclComm_t>(c));
            if (r != ncclSuccess && r != ncclInProgress && first == ncclSuccess) {
                first = r;
            }
        }
        const ncclResult_t end = ncclGroupEnd();
        NcclCheck(first, "ncclCommFinalize");
        NcclCheck(end, "ncclGroupEnd(finalize)", true);
        CommSettle(live.data(), live.size(), "ncclCommFinalize", nullptr, 10.0);
    } catch (...) {
        ok = false;
    }
    if (!ok) {
        CommAbortAll(live);
        return;
    }
    std::vector<void*> stuck;
    for (void* c : live) {
        if (ncclCommDestroy(static_cast<ncclComm_t>(c)) != ncclSuccess) {
            stuck.push_back(c);
        }
    }
    CommAbortAll(stuck);
}

Injection Injection::FromEnv() {
    Injection in;
    const char* v = std::getenv("SRT_ENGINE_INJECT");
    if (v == nullptr || *v == '\0') {
        return in;
    }
    const std::string s(v);
    const std::size_t a = s.find(':'), b = a == std::string::npos ? a : s.find(':', a + 1);
    if (b == std::string::npos) {
        throw std::runtime_error("SRT_ENGINE_INJECT must be fail:<local>:<batch> or stall:<local>:<batch>");
    }
    const std::string kind = s.substr(0, a);
    in.kind = kind == "fail" ? kFail : kind == "stall" ? kStall : kNone;
    if (in.kind == kNone) {
        throw std::runtime_error("SRT_ENGINE_INJECT: unknown kind '" + kind + "'");
    }
    in.local = static_cast<std::size_t>(std::strtoul(s.c_str() + a + 1, nullptr, 10));
    in.batch = static_cast<std::size_t>(std::strtoul(s.c_str() + b + 1, nullptr, 10));
    return in;
}

}  // namespace srt
