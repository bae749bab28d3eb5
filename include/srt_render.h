/*
 * srt_render.h -- extension C ABI of libModelRunner.so (not part of the reference ABI).
 *
 * The reference exposes only the 14 ml* entry points of model_runner.h, which take host
 * images. Benchmarks, parity tests and multi-process (one rank per GPU) callers need the
 * render stages on device-resident buffers and a way to produce scene files; that is this
 * header. Plain pointers and sizes only; `stream` is a hipStream_t passed as void*.
 * Every int-returning function returns 0 on success, -1 on failure; the failure text is
 * then available from srtGetLastError() (thread-local).
 */
#ifndef SRT_RENDER_H
#define SRT_RENDER_H

#include <stddef.h>

#include "model_runner.h" /* ML_API_ENTRY */

#ifdef __cplusplus
extern "C" {
#endif

/* Scene kinds for srtWriteScene (DESIGN.md "Scene file"). */
#define SRT_SCENE_TRIANGLE 0 /* one triangle: config C1 */
#define SRT_SCENE_CORNELL 1  /* 12-triangle Cornell box: config C2 */
#define SRT_SCENE_SOUP 2     /* synthetic soup: configs C3-C5 */

/* Trace kernel variants for srtTraceAsync. */
#define SRT_TRACE_LDS 0
#define SRT_TRACE_SCALAR 1
#define SRT_TRACE_CULL 2 /* hierarchical block/lane/ray cull; bit-identical output */
#define SRT_TRACE_BVH 3  /* screen-space 8-wide BVH, wave-packet traversal; bit-identical output */

ML_API_ENTRY const char* srtGetLastError(void);

/* Write a generated scene file. `triangles`, `seed` and `size` (soup half-extent, 0 =
 * default 0.02 below 1M triangles, 0.01 from 1M) apply to SRT_SCENE_SOUP only. */
ML_API_ENTRY int srtWriteScene(const char* path, int kind, unsigned long long triangles,
                               unsigned long long seed, float size);

/* Read a scene file's triangle count. */
ML_API_ENTRY int srtSceneTriangles(const char* path, unsigned long long* triangles);

/* Load a scene file (binary, or Wavefront OBJ when the path ends in ".obj") and copy its
 * contents out: vertices (triangles x 9 floats), albedo (triangles x 3), camera (10 floats:
 * eye, lookat, up, vfov_deg), background (3) and the header flags (data types of the model's
 * images, 1 = FLOAT16 output, 2 = FLOAT16 input). Any output pointer may be NULL; `capacity`
 * is the number of triangles the vertex / albedo arrays hold (fewer than the scene's: fail). */
ML_API_ENTRY int srtReadScene(const char* path, unsigned long long capacity, unsigned long long* triangles,
                              float* vertices, float* albedo, float* camera10, float* background3,
                              unsigned* flags);

/* Load src_path (binary or OBJ) and write it as a binary scene file to dst_path, with the
 * data types of the model's images set: input_dtype / output_dtype = ML_FLOAT32 or
 * ML_FLOAT16, or -1 to keep the source's. */
ML_API_ENTRY int srtConvertScene(const char* src_path, const char* dst_path, int input_dtype, int output_dtype);

/* Affine primary-ray frame of a scene at W x H: 12 floats origin[3] base[3] du[3] dv[3]. */
ML_API_ENTRY int srtSceneFrame(const char* path, size_t width, size_t height, float* frame12);

/* Device-resident scene (vertices, albedo, edge records) on one HIP device. */
typedef struct srt_device_scene_t* srt_device_scene;

ML_API_ENTRY srt_device_scene srtDeviceSceneCreate(const char* path, int device);
ML_API_ENTRY void srtDeviceSceneRelease(srt_device_scene scene);
ML_API_ENTRY unsigned long long srtDeviceSceneTriangles(srt_device_scene scene);

/* The scene's spatial order, built on the device at load (ids sorted by the Morton code of their
 * centroid's image-plane position under the scene camera; rocPRIM radix sort): copied to
 * `order` (capacity entries, NULL = skip) and the build's device time in ms (NULL = skip). */
ML_API_ENTRY int srtDeviceSceneOrder(srt_device_scene scene, unsigned* order, unsigned long long capacity,
                                     double* build_ms);

/* Stage 1: edge-record setup for a W x H frame (one thread per triangle). The work is
 * enqueued by the next srtTraceAsync, on that call's stream, fused into its first kernel; the
 * records then serve every srtTraceAsync until the next srtPrepareAsync. */
ML_API_ENTRY int srtPrepareAsync(srt_device_scene scene, size_t width, size_t height, void* stream);

/* Stage 2: trace frame rows [row_begin, row_begin + row_count) of the prepared frame.
 * d_offsets: row_count x width x 2 float (sample offsets, band-local rows);
 * d_rgba:    row_count x width x 4 float (r, g, b, float(tri_id)). */
ML_API_ENTRY int srtTraceAsync(srt_device_scene scene, const float* d_offsets, float* d_rgba,
                               size_t row_begin, size_t row_count, int variant, void* stream);

/* Stage 2 for deferred shading: the same trace, storing only each pixel's hit triangle id
 * (-1 = miss) into d_ids (row_count x width int32, band-local rows); 4 B per pixel instead of 16,
 * the payload a multi-GPU band gather moves. */
ML_API_ENTRY int srtTraceIdsAsync(srt_device_scene scene, const float* d_offsets, int* d_ids,
                                  size_t row_begin, size_t row_count, int variant, void* stream);

/* Stages 1-2 for a batch of up to SRT_MAX_BATCH frames of the prepared camera (same band of
 * each): frame f's sample offsets d_offsets[f] (row_count x width x 2, band-local) and either its
 * RGBA d_rgba[f] (row_count x width x 4) or, with d_rgba NULL, its hit ids d_ids[f]
 * (row_count x width). Every frame gets the whole per-frame work of srtPrepareAsync +
 * srtTraceAsync (record setup, bins, trace): the same pixels, bit for bit; the cull variant runs
 * the batch with one launch per stage, so a frame costs a quarter of the host launches.
 * row_interleave 1: the band is frame rows [row_begin, row_begin + row_count). P > 1: the frame's
 * 16-row tile rows are dealt round-robin to P bands and this band holds tile rows
 * row_begin / 16 + k P, k = 0, 1, ..., concatenated (row_begin a multiple of 16, row_count =
 * those rows' total; SRT_TILE_ROWS = 16). */
#define SRT_MAX_BATCH 8
#define SRT_TILE_ROWS 16
ML_API_ENTRY int srtTraceBatchAsync(srt_device_scene scene, const float* const* d_offsets, float* const* d_rgba,
                                    int* const* d_ids, size_t frames, size_t row_begin, size_t row_count,
                                    size_t row_interleave, int variant, void* stream);

/* Stage 3 (deferred shading): rows [row_begin, row_begin + row_count) of the prepared frame
 * shaded from hit ids (as srtTraceIdsAsync writes them) and sample offsets (both band-local,
 * row_count x width) into d_rgba: bit-identical to srtTraceAsync's RGBA. */
ML_API_ENTRY int srtShadeAsync(srt_device_scene scene, const float* d_offsets, const int* d_ids, float* d_rgba,
                               size_t row_begin, size_t row_count, void* stream);

/* Stage 3 for a batch of `frames` frames of the prepared camera (the multi-process band path,
 * where one gather carries several frames): the ids arrive band-major, as a gather of every
 * rank's (frames x band_rows x width) band buffer leaves them,
 *   d_ids[band][frame][band_rows][width],
 * with bands = ceil(height / band_rows) contiguous bands (interleaved = 0), or `interleaved`
 * bands that took the frame's 16-row tile rows round-robin (srtTraceBatchAsync row_interleave;
 * band_rows >= the largest band's rows). d_offsets is the frame's (height x width x 2), d_rgba
 * receives frames x height x width x 4. One launch; each frame is bit-identical to
 * srtTraceAsync's RGBA. */
ML_API_ENTRY int srtShadeBandsAsync(srt_device_scene scene, const float* d_offsets, const int* d_ids, float* d_rgba,
                                    size_t frames, size_t band_rows, size_t interleaved, void* stream);

/* Calls on one srt_device_scene are ordered: the per-frame edge records and the cull work
 * buffer are shared, so a call on a different stream than the previous call first waits (HIP
 * event) for the work enqueued before it. Use one scene per stream for concurrent frames. */

/* Stage timing (measurement): while enabled, srtPrepareAsync and srtTraceAsync bind HIP events
 * to their kernels' own dispatch packets (hipExtLaunchKernelGGL start/stop events: no extra
 * packets on the stream). srtTakeStageTimes waits for them, writes the number of timed trace
 * calls and the mean milliseconds of the prepare kernel, the bin stage (TileInfo start to
 * TileOrder end; 0 for variants without one) and the trace kernel alone, and forgets them. */
ML_API_ENTRY int srtSetStageTiming(srt_device_scene scene, int enable);
ML_API_ENTRY int srtTakeStageTimes(srt_device_scene scene, unsigned* launches, double* prepare_ms, double* bin_ms,
                                   double* trace_ms);

/* ---------------------------------------------------------------------------------------------
 * Frame engine (csrc/engine.h): a stream of frames over one or more GPUs, the native multi-GPU
 * path of BASELINE config C4 (and C3 / C5 on one GPU). A run is a sequence of batches of `batch`
 * frames; every device keeps `queues` batches in flight (own scene buffers and HIP stream each).
 * Split SRT_SPLIT_BANDS over P devices: each frame is cut into P row bands (the frame's 16-row tile
 * rows dealt round-robin, or contiguous blocks), device d traces band d (hit ids, 4 B per pixel),
 * the bands move over RCCL to the frame's compositor, which shades the frame from the ids (one
 * launch per batch, bit-identical to the fused trace). Exchanges: SRT_EXCHANGE_ALLTOALL (frame f of
 * a batch composited on device f % P; the batch's P gathers fused into one ncclSend / ncclRecv
 * group), SRT_EXCHANGE_ROTATING (the batch gathered to device b % P), SRT_EXCHANGE_ROOT (device 0),
 * SRT_EXCHANGE_SHARE (frame f composited on device c = f % P, which traces `share` of every
 * share + P - 1 tile rows of it itself, straight into the frame; each other device traces one tile
 * row per such cycle and sends its ids: the exchange and the shading shrink to (P - 1) / (share +
 * P - 1) of a frame; interleaved rows only; bench.py's default).
 * P == 1: trace + shade fused (RGBA). SRT_SPLIT_FRAMES: every device renders whole frames of its
 * own (no exchange). Devices: all in this process (srtEngineCreate; one worker thread per device,
 * ncclCommInitAll; a repeated device exchanges by device copies -- the one-GPU rehearsal), or one
 * per process (srtEngineCreateRank; ncclCommInitRank with a unique id from srtEngineUniqueId). */
typedef struct srt_engine_t* srt_engine;
#define SRT_ROWS_INTERLEAVED 0
#define SRT_ROWS_CONTIGUOUS 1
#define SRT_ROWS_ROTATED 2 /* contiguous bands, device p tracing band (p + c) % P of a frame composited on
                              device c (SRT_EXCHANGE_ALLTOALL): even load, one block of rows per band; over
                              two devices the compositor's own band 0 takes env SRT_ROTATE_OWN per cent of
                              the frame (default 80, 50 = halves): only band 1 crosses the one link */
#define SRT_EXCHANGE_ALLTOALL 0
#define SRT_EXCHANGE_ROTATING 1
#define SRT_EXCHANGE_ROOT 2
#define SRT_EXCHANGE_SHARE 3
#define SRT_SPLIT_BANDS 0
#define SRT_SPLIT_FRAMES 1
/* srt_engine_options.flags */
#define SRT_ENGINE_RCCL_SELF 1 /* one device: the bands path with the ids sent to itself over a one-rank
                                  RCCL communicator (the real exchange, waits and abort on one GPU) */
typedef struct srt_engine_options {
    size_t struct_size; /* sizeof(srt_engine_options) as the caller was compiled (checked: a caller built
                           against another layout is refused, never read past its struct) */
    int variant;    /* SRT_TRACE_* */
    size_t queues;  /* batches in flight per device (0 = 2) */
    size_t batch;   /* frames per batch (0 = 16) */
    int rows;       /* SRT_ROWS_* */
    int exchange;   /* SRT_EXCHANGE_* */
    int split;      /* SRT_SPLIT_* */
    int simulate;   /* measurement: srtEngineCreateRank without peers, the exchange skipped (0 = off) */
    size_t launch;  /* frames per trace launch, <= 256 (0 = env SRT_LAUNCH_FRAMES, else 8 for whole
                       frames, 64 for bands over more than one device) */
    int flags;      /* SRT_ENGINE_* bits (0 = none) */
    size_t share;   /* SRT_EXCHANGE_SHARE: the compositor's tile rows per cycle, a power of two (0 = srtShareAuto) */
    size_t own_rows; /* SRT_ROWS_ROTATED over two devices: rows of the compositor's own band 0 (0 = env
                        SRT_ROTATE_OWN if set, else derived from the link measured at creation when RCCL
                        joins distinct devices -- srtRotateSplitForLink --, else 80 % of the frame) */
} srt_engine_options;

/* 128-byte RCCL unique id for srtEngineCreateRank (call on one rank, share with the others). */
ML_API_ENTRY int srtEngineUniqueId(void* id128);
ML_API_ENTRY srt_engine srtEngineCreate(const char* scene_path, const int* devices, size_t device_count, size_t width,
                                        size_t height, const srt_engine_options* options);
/* Every rank calls this concurrently (RCCL communicator setup synchronises them).
 * Failures: communicators are nonblocking and every wait behind RCCL is polled with a deadline (env
 * SRT_COMM_TIMEOUT_S, default 60 s); when a device's worker fails, or no device progresses for that
 * long, every communicator is aborted (ncclCommAbort) and srtEngineRun returns -1 with the first
 * error in srtGetLastError -- never a hang. The engine then refuses further work. */
ML_API_ENTRY srt_engine srtEngineCreateRank(const char* scene_path, int device, int rank, int world,
                                            const void* unique_id128, size_t width, size_t height,
                                            const srt_engine_options* options);
ML_API_ENTRY void srtEngineRelease(srt_engine engine);
/* `count` full-frame sample-offset images (count x height x width x 2 floats, host), kept resident on
 * every device; frame k reads input k % count. */
ML_API_ENTRY int srtEngineSetInputs(srt_engine engine, const float* host_offsets, size_t count);
/* Render `batches` x batch frames, continuing the frame sequence; synchronous. */
ML_API_ENTRY int srtEngineRun(srt_engine engine, size_t batches);
/* The locally composited frames of each queue's last batch (up to 4 per queue) vs a single-device
 * full-frame render of their inputs (another trace variant), bit for bit: mismatching and checked
 * frame counts. */
ML_API_ENTRY int srtEngineVerify(srt_engine engine, size_t* mismatches, size_t* checked);
/* Frame k of the last `queues` batches into host RGBA (height x width x 4 floats); fails when another
 * rank composited it (bands) or it is no longer resident. */
ML_API_ENTRY int srtEngineReadFrame(srt_engine engine, size_t frame, float* host_rgba);
/* Stage times of `launches` single-frame traces of local device `local`'s band (see
 * srtTakeStageTimes). */
ML_API_ENTRY int srtEngineStageTimes(srt_engine engine, size_t local, size_t launches, unsigned* launched,
                                     double* prepare_ms, double* bin_ms, double* trace_ms);
/* The same for launches of `frames` frames each (1 .. batch): one launch per stage for all of them,
 * one launch in flight; the times are per launch. */
ML_API_ENTRY int srtEngineStageTimesBatch(srt_engine engine, size_t local, size_t launches, size_t frames,
                                          unsigned* launched, double* prepare_ms, double* bin_ms, double* trace_ms);
/* Host self-test of the engine's worker pool failure handling (no device): `workers` workers, worker
 * `failing` throws (mode 1) or stalls (mode 2) while every other worker waits for a release only the
 * abort gives. Writes the error the run ended with into msg (truncated to msg_size - 1), the seconds
 * it took and how often the abort hook ran. */
ML_API_ENTRY int srtEnginePoolSelfTest(size_t workers, size_t failing, int mode, double timeout_s, double* elapsed_s,
                                       int* abort_calls, char* msg, size_t msg_size);
/* SRT_EXCHANGE_SHARE's default tile rows per cycle for a frame of `height` rows over `devices`
 * devices: the largest power of two <= 32 with share + devices - 1 <= ceil(height / 16). */
ML_API_ENTRY size_t srtShareAuto(size_t height, size_t devices);
/* SRT_ROWS_ROTATED over two devices without a measured link: rows of the compositor's own band 0 for a
 * frame of `height` rows (env SRT_ROTATE_OWN, an integer per cent in 1..99, default 80, rounded to 16-row
 * tile rows, within [1, height - 1]); 0 with srtGetLastError set when SRT_ROTATE_OWN is not such an integer. */
ML_API_ENTRY size_t srtRotateOwnRows(size_t height);
/* The two-device split an engine derives from its link: for a link of `link_gbs`
 * GB/s per direction, a one-GPU frame time of `frame_us` microseconds and an exchange payload of
 * `bytes_per_pixel`, the smallest own band -- whole 16-row tile rows, at least half the frame -- whose
 * link time per frame of the job, (height - rows) x width x bytes_per_pixel / 2 / rate, stays within
 * 80 % of the GPUs' time per frame of the job, frame_us x (0.553 + 0.25 (height - rows) / height); the
 * largest own band (one tile row sent) when none does. */
ML_API_ENTRY size_t srtRotateSplitForLink(size_t height, size_t width, double link_gbs, double frame_us,
                                          double bytes_per_pixel);
/* The engine's two-device split: own band rows (0 unless rotated bands over two devices), the band
 * buffers' rows, the link rate measured at creation (GB/s per direction of the slowest device: RCCL
 * send / receive groups of 32 MB; 0 without RCCL), the one-GPU frame time measured for the split (us; 0
 * when not derived), and the source: 0 none, 1 the option, 2 env SRT_ROTATE_OWN, 3 the measured link,
 * 4 the 80 % default. One rank per process: the ranks' splits are compared at creation (a mismatch fails
 * the create). */
ML_API_ENTRY int srtEngineSplit(srt_engine engine, size_t* own_rows, size_t* buffer_rows, double* link_gbs,
                                double* frame_us, int* source);
/* Shape of the run: devices in the job, local devices, rows of local device 0's band, rows of every
 * band buffer, whether the exchange uses RCCL, exchanged bytes per frame (bands, all devices). */
ML_API_ENTRY int srtEngineInfo(srt_engine engine, size_t* devices, size_t* local_devices, size_t* band_rows,
                               size_t* buffer_rows, int* rccl, double* exchange_bytes_per_frame);
/* The last srtEngineRun's exchange on local device `local`: every batch's send / receive group (RCCL)
 * or copies (device copies) timed by HIP events on the device's exchange stream -- groups timed, mean
 * ms per group (from the stream reaching the group to its completion: peers' lateness included), and
 * the bytes the device sent per group. Zero groups without an exchange. */
ML_API_ENTRY int srtEngineExchangeStats(srt_engine engine, size_t local, size_t* groups, double* ms_mean,
                                        double* bytes_sent);
/* Host self-test of the engine's exchange layout (no device): band_ids[d] = band d's hit ids of a
 * batch's frames (batch x buffer rows x width int32, buffer rows = srtEngineInfo's); recv[c]
 * receives compositor c's buffer as the device path lays it out, [bands][frames of c][buffer rows]
 * [width] (frames of c: recv_frames[c]; pass NULL recv to only query recv_frames). */
ML_API_ENTRY int srtExchangeHost(const int* const* band_ids, size_t bands, size_t width, size_t height, int rows,
                                 int exchange, size_t batch, size_t batch_index, int* const* recv,
                                 size_t* recv_frames, size_t* buffer_rows);
/* The same for SRT_EXCHANGE_SHARE at `share` tile rows per cycle (0 = srtShareAuto): band_ids[d] =
 * device d's traced ids of the batch's frames (batch x buffer rows x width int32, buffer rows = one
 * class of share + bands - 1 interleaved classes): of frame f its sender class (share + (d - c - 1)
 * mod bands for compositor c = f % bands; unused when d = c); recv[c]: [bands][frames of c][buffer
 * rows][width], sender d at slot (d - c - 1) mod bands (slot bands - 1: unused). */
ML_API_ENTRY int srtExchangeHostShare(const int* const* band_ids, size_t bands, size_t width, size_t height,
                                      size_t share, size_t batch, size_t batch_index, int* const* recv,
                                      size_t* recv_frames, size_t* buffer_rows);
/* Host self-test of a record's screen box (render.hip ComputeRecord): c = the
 * 9 edge coefficients (c0A, cxA, cyA, c0B, cxB, cyB, c0C, cxC, cyC); mode 0 = the float fast path
 * where it applies, else the double solve (what the kernels do), 1 = the double solve, 2 = the fast
 * path only. box = (xlo, xhi, ylo, yhi). Returns 0, or -1 with mode 2 where the fast path does
 * not apply. */
ML_API_ENTRY int srtScreenBoxHost(const float* c, int mode, float* box);

#ifdef __cplusplus
}
#endif

#endif /* SRT_RENDER_H */
