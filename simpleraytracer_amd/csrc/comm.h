// RCCL communicators and waits that end in an error, never a hang.
//
// The reference turns every failure into a status plus a cached message (ML_FAIL / ML_INVALID_HANDLE,
// model_runner/context.cpp:40-48, model.cpp:161-294); a multi-GPU render must do the same when one
// device (or one rank) stops: a peer that never posts its ncclSend leaves the receiver's RCCL kernel
// waiting forever, and a plain hipStreamSynchronize behind it never returns.
//
// So every communicator here is created NONBLOCKING (ncclConfig_t::blocking = 0): RCCL calls return
// at once (ncclInProgress while their enqueue or connection setup continues in the background) and
// their progress is polled with ncclCommGetAsyncError. Every wait on work queued behind RCCL polls
// its HIP event, the communicators' async errors, an abort flag and a deadline. On any failure the
// owner aborts every communicator (ncclCommAbort: kernels waiting on a peer see the abort flag and
// exit, so the streams drain) and rethrows the first error.
//
// Threads: the owner's workers touch the communicators only under CommCtl::mu (shared) and only
// while CommCtl::abort is false; the owner sets `abort` first, then takes `mu` exclusively to call
// ncclCommAbort (which frees the communicators). No RCCL call on a nonblocking communicator blocks,
// so the exclusive lock is granted within microseconds.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <cstddef>
#include <shared_mutex>
#include <string>
#include <vector>

namespace srt {

// Seconds a wait may go without completing before it fails: env SRT_COMM_TIMEOUT_S (default 60).
double CommTimeoutSeconds();

// What the waits share with their owner: the abort flag they poll, a progress counter they bump, and
// the lock under which they touch the communicators.
struct CommCtl {
    std::atomic<bool> abort{false};
    std::atomic<unsigned long> progress{0};
    std::shared_mutex mu;
};

// Throws std::runtime_error("RCCL error: <what>: <reason>") unless res is ncclSuccess, or
// ncclInProgress when `in_progress_ok` (a call on a nonblocking communicator).
void NcclCheck(ncclResult_t res, const char* what, bool in_progress_ok = false);

// Waits until none of `comms` reports ncclInProgress (a nonblocking init, group end or finalize has
// finished its host-side work). Throws on an async error, on ctl->abort, or after `timeout_s`
// seconds (<= 0: CommTimeoutSeconds()).
void CommSettle(void* const* comms, std::size_t n, const char* what, CommCtl* ctl = nullptr, double timeout_s = 0.0);

// Nonblocking communicators over `devices` (all in this process, rank i on devices[i]; the
// ncclCommInitAll of a nonblocking world), settled.
std::vector<void*> CommInitAll(const std::vector<int>& devices);
// This process's rank of a `world`-rank nonblocking communicator on `device`, settled.
void* CommInitRank(int device, int world, const void* unique_id128, int rank);

// Polls `ev` until it has completed. Throws on an async error of any of `comms`, on ctl->abort, or
// when `timeout_s` (<= 0: CommTimeoutSeconds()) passes without completion; bumps ctl->progress
// when the event completes.
void CommWaitEvent(hipEvent_t ev, void* const* comms, std::size_t n, const char* what, CommCtl* ctl = nullptr,
                   double timeout_s = 0.0);

// hipStreamSynchronize with a deadline (never throws): false when the stream did not drain in
// `timeout_s` seconds or reported an error.
bool StreamDrain(hipStream_t stream, double timeout_s) noexcept;

// ncclCommAbort on every communicator (it also frees them), then clears the list.
void CommAbortAll(std::vector<void*>& comms) noexcept;
// Orderly teardown: ncclCommFinalize + settle + ncclCommDestroy on each; a communicator that does
// not finish within the timeout is aborted instead. Clears the list.
void CommDestroyAll(std::vector<void*>& comms) noexcept;

// Failure injection for the abort tests (env SRT_ENGINE_INJECT="fail:<local>:<batch>" -- that
// worker throws before tracing batch <batch> --, or "stall:<local>:<batch>" -- it stops making
// progress there, like a worker stuck behind a dead peer, until the run is aborted).
struct Injection {
    enum Kind { kNone = 0, kFail = 1, kStall = 2 };
    int kind = kNone;
    std::size_t local = 0, batch = 0;
    static Injection FromEnv();
};

}  // namespace srt
