// Extension C entry points (include/srt_render.h): scene files and device-level stages.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <exception>
#include <string>
#include <vector>

#include "cpu_render.h"
#include "engine.h"
#include "render.h"
#include "renderer.h"
#include "scene.h"
#include "srt_render.h"

namespace {

thread_local std::string g_last_error;

template <class F>
int Guarded(F&& f) {
    try {
        f();
        g_last_error.clear();
        return 0;
    } catch (std::exception& e) {
        g_last_error = e.what();
    } catch (...) {
        g_last_error = "unknown error";
    }
    return -1;
}

srt::DeviceScene* FromHandle(srt_device_scene s) { return reinterpret_cast<srt::DeviceScene*>(s); }

// Binds the scene's device for the duration of a call, restoring the caller's device.
class Bind {
public:
    explicit Bind(int device) {
        if (hipGetDevice(&m_prev) != hipSuccess) {
            m_prev = -1;
        }
        srt::HipCheck(hipSetDevice(device), "hipSetDevice");
    }
    ~Bind() {
        if (m_prev >= 0) {
            (void)hipSetDevice(m_prev);
        }
    }

private:
    int m_prev = -1;
};

}  // namespace

extern "C" {

ML_API_ENTRY const char* srtGetLastError(void) { return g_last_error.c_str(); }

ML_API_ENTRY int srtWriteScene(const char* path, int kind, unsigned long long triangles, unsigned long long seed,
                               float size) {
    return Guarded([&] {
        if (path == nullptr) {
            throw std::runtime_error("Bad path argument");
        }
        srt::SaveScene(srt::MakeScene(kind, triangles, seed, size), path);
    });
}

ML_API_ENTRY int srtSceneTriangles(const char* path, unsigned long long* triangles) {
    return Guarded([&] {
        if (path == nullptr || triangles == nullptr) {
            throw std::runtime_error("Bad argument");
        }
        *triangles = srt::LoadScene(path).triangle_count();
    });
}

ML_API_ENTRY int srtReadScene(const char* path, unsigned long long capacity, unsigned long long* triangles,
                              float* vertices, float* albedo, float* camera10, float* background3,
                              unsigned* flags) {
    return Guarded([&] {
        if (path == nullptr) {
            throw std::runtime_error("Bad path argument");
        }
        const srt::Scene s = srt::LoadScene(path);
        const unsigned long long n = s.triangle_count();
        if (triangles != nullptr) {
            *triangles = n;
        }
        if ((vertices != nullptr || albedo != nullptr) && capacity < n) {
            throw std::runtime_error("Buffer too small: " + std::to_string(capacity) + " triangles for " +
                                     std::to_string(n));
        }
        if (vertices != nullptr) {
            std::copy(s.vertices.begin(), s.vertices.end(), vertices);
        }
        if (albedo != nullptr) {
            std::copy(s.albedo.begin(), s.albedo.end(), albedo);
        }
        if (camera10 != nullptr) {
            std::copy(s.camera.eye, s.camera.eye + 3, camera10);
            std::copy(s.camera.lookat, s.camera.lookat + 3, camera10 + 3);
            std::copy(s.camera.up, s.camera.up + 3, camera10 + 6);
            camera10[9] = s.camera.vfov_deg;
        }
        if (background3 != nullptr) {
            std::copy(s.background, s.background + 3, background3);
        }
        if (flags != nullptr) {
            *flags = s.flags;
        }
    });
}

ML_API_ENTRY int srtConvertScene(const char* src_path, const char* dst_path, int input_dtype, int output_dtype) {
    return Guarded([&] {
        if (src_path == nullptr || dst_path == nullptr) {
            throw std::runtime_error("Bad path argument");
        }
        srt::Scene s = srt::LoadScene(src_path);
        auto set = [&](int dtype, std::uint32_t bit, const char* what) {
            if (dtype == -1) {
                return;
            }
            if (dtype != ML_FLOAT32 && dtype != ML_FLOAT16) {
                throw std::runtime_error(std::string("Bad ") + what + " data type " + std::to_string(dtype));
            }
            s.flags = dtype == ML_FLOAT16 ? (s.flags | bit) : (s.flags & ~bit);
        };
        set(input_dtype, srt::kFlagInputFloat16, "input");
        set(output_dtype, srt::kFlagOutputFloat16, "output");
        srt::SaveScene(s, dst_path);
    });
}

ML_API_ENTRY int srtSceneFrame(const char* path, size_t width, size_t height, float* frame12) {
    return Guarded([&] {
        if (path == nullptr || frame12 == nullptr || width == 0 || height == 0) {
            throw std::runtime_error("Bad argument");
        }
        const srt::Frame f = srt::MakeFrame(srt::LoadScene(path).camera, width, height);
        for (int k = 0; k < 3; ++k) {
            frame12[k] = f.origin[k];
            frame12[3 + k] = f.base[k];
            frame12[6 + k] = f.du[k];
            frame12[9 + k] = f.dv[k];
        }
    });
}

ML_API_ENTRY srt_device_scene srtDeviceSceneCreate(const char* path, int device) {
    srt::DeviceScene* out = nullptr;
    Guarded([&] {
        if (path == nullptr) {
            throw std::runtime_error("Bad path argument");
        }
        const srt::Scene scene = srt::LoadScene(path);
        int count = 0;
        if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count) {
            throw std::runtime_error("HIP error: device " + std::to_string(device) + " not available (" +
                                     std::to_string(count) + " present); the device stages have no CPU path (ml* renders on the CPU with ML_VISIBLE_DEVICES=cpu)");
        }
        out = new srt::DeviceScene(scene, device);
    });
    return reinterpret_cast<srt_device_scene>(out);
}

ML_API_ENTRY void srtDeviceSceneRelease(srt_device_scene scene) { delete FromHandle(scene); }

ML_API_ENTRY unsigned long long srtDeviceSceneTriangles(srt_device_scene scene) {
    return scene == nullptr ? 0ULL : FromHandle(scene)->triangles();
}

ML_API_ENTRY int srtDeviceSceneOrder(srt_device_scene scene, unsigned* order, unsigned long long capacity,
                                     double* build_ms) {
    return Guarded([&] {
        if (scene == nullptr) {
            throw std::runtime_error("Bad scene handle");
        }
        srt::DeviceScene* s = FromHandle(scene);
        if (order != nullptr) {
            if (capacity < s->triangles()) {
                throw std::runtime_error("Buffer too small: " + std::to_string(capacity) + " entries for " +
                                         std::to_string(s->triangles()));
            }
            Bind bind(s->device());
            srt::HipCheck(hipMemcpy(order, s->order(), s->triangles() * sizeof(unsigned), hipMemcpyDeviceToHost),
                          "hipMemcpy(order)");
        }
        if (build_ms != nullptr) {
            *build_ms = s->build_ms();
        }
    });
}

ML_API_ENTRY int srtPrepareAsync(srt_device_scene scene, size_t width, size_t height, void* stream) {
    return Guarded([&] {
        if (scene == nullptr) {
            throw std::runtime_error("Bad scene handle");
        }
        srt::DeviceScene* s = FromHandle(scene);
        Bind bind(s->device());
        s->Prepare(width, height, static_cast<hipStream_t>(stream));
    });
}

ML_API_ENTRY int srtTraceAsync(srt_device_scene scene, const float* d_offsets, float* d_rgba, size_t row_begin,
                               size_t row_count, int variant, void* stream) {
    return Guarded([&] {
        if (scene == nullptr) {
            throw std::runtime_error("Bad scene handle");
        }
        if ((d_offsets == nullptr || d_rgba == nullptr) && row_count != 0) {
            throw std::runtime_error("Bad buffer argument");
        }
        if (variant != SRT_TRACE_LDS && variant != SRT_TRACE_SCALAR && variant != SRT_TRACE_CULL &&
            variant != SRT_TRACE_BVH) {
            throw std::runtime_error("Unknown trace variant " + std::to_string(variant));
        }
        srt::DeviceScene* s = FromHandle(scene);
        Bind bind(s->device());
        s->Trace(d_offsets, d_rgba, row_begin, row_count, variant, static_cast<hipStream_t>(stream));
    });
}

ML_API_ENTRY int srtTraceIdsAsync(srt_device_scene scene, const float* d_offsets, int* d_ids, size_t row_begin,
                                  size_t row_count, int variant, void* stream) {
    return Guarded([&] {
        if (scene == nullptr) {
            throw std::runtime_error("Bad scene handle");
        }
        if ((d_offsets == nullptr || d_ids == nullptr) && row_count != 0) {
            throw std::runtime_error("Bad buffer argument");
        }
        if (variant != SRT_TRACE_LDS && variant != SRT_TRACE_SCALAR && variant != SRT_TRACE_CULL &&
            variant != SRT_TRACE_BVH) {
            throw std::runtime_error("Unknown trace variant " + std::to_string(variant));
        }
        srt::DeviceScene* s = FromHandle(scene);
        Bind bind(s->device());
        s->Trace(d_offsets, nullptr, row_begin, row_count, variant, static_cast<hipStream_t>(stream), d_ids);
    });
}

static_assert(SRT_MAX_BATCH == srt::kMaxBatch, "include/srt_render.h SRT_MAX_BATCH");
static_assert(SRT_TILE_ROWS == srt::kCullTileRows, "include/srt_render.h SRT_TILE_ROWS");

ML_API_ENTRY int srtTraceBatchAsync(srt_device_scene scene, const float* const* d_offsets, float* const* d_rgba,
                                    int* const* d_ids, size_t frames, size_t row_begin, size_t row_count,
                                    size_t row_interleave, int variant, void* stream) {
    return Guarded([&] {
        if (scene == nullptr) {
            throw std::runtime_error("Bad scene handle");
        }
        if (frames > SRT_MAX_BATCH) {
            throw std::runtime_error("At most " + std::to_string(SRT_MAX_BATCH) + " frames per batch");
        }
        if (frames != 0 && row_count != 0) {
            if (d_offsets == nullptr || (d_rgba == nullptr) == (d_ids == nullptr)) {
                throw std::runtime_error("Bad buffer argument");
            }
            for (size_t f = 0; f < frames; ++f) {
                if (d_offsets[f] == nullptr || (d_rgba != nullptr ? d_rgba[f] == nullptr : d_ids[f] == nullptr)) {
                    throw std::runtime_error("Bad buffer argument");
                }
            }
        }
        if (variant != SRT_TRACE_LDS && variant != SRT_TRACE_SCALAR && variant != SRT_TRACE_CULL &&
            variant != SRT_TRACE_BVH) {
            throw std::runtime_error("Unknown trace variant " + std::to_string(variant));
        }
        srt::DeviceScene* s = FromHandle(scene);
        Bind bind(s->device());
        s->TraceBatch(d_offsets, d_rgba, d_ids, frames, row_begin, row_count, variant, static_cast<hipStream_t>(stream),
                      row_interleave);
    });
}

ML_API_ENTRY int srtShadeAsync(srt_device_scene scene, const float* d_offsets, const int* d_ids, float* d_rgba,
                               size_t row_begin, size_t row_count, void* stream) {
    return Guarded([&] {
        if (scene == nullptr) {
            throw std::runtime_error("Bad scene handle");
        }
        if ((d_offsets == nullptr || d_ids == nullptr || d_rgba == nullptr) && row_count != 0) {
            throw std::runtime_error("Bad buffer argument");
        }
        srt::DeviceScene* s = FromHandle(scene);
        Bind bind(s->device());
        s->Shade(d_offsets, d_ids, d_rgba, row_begin, row_count, static_cast<hipStream_t>(stream));
    });
}

ML_API_ENTRY int srtShadeBandsAsync(srt_device_scene scene, const float* d_offsets, const int* d_ids, float* d_rgba,
                                    size_t frames, size_t band_rows, size_t interleaved, void* stream) {
    return Guarded([&] {
        if (scene == nullptr) {
            throw std::runtime_error("Bad scene handle");
        }
        if ((d_offsets == nullptr || d_ids == nullptr || d_rgba == nullptr) && frames != 0) {
            throw std::runtime_error("Bad buffer argument");
        }
        if (band_rows == 0) {
            throw std::runtime_error("band_rows must be positive");
        }
        srt::DeviceScene* s = FromHandle(scene);
        Bind bind(s->device());
        s->Shade(d_offsets, d_ids, d_rgba, 0, s->height(), static_cast<hipStream_t>(stream), frames, band_rows,
                 interleaved);
    });
}

ML_API_ENTRY int srtSetStageTiming(srt_device_scene scene, int enable) {
    return Guarded([&] {
        if (scene == nullptr) {
            throw std::runtime_error("Bad scene handle");
        }
        FromHandle(scene)->SetTiming(enable != 0);
    });
}

ML_API_ENTRY int srtTakeStageTimes(srt_device_scene scene, unsigned* launches, double* prepare_ms, double* bin_ms,
                                   double* trace_ms) {
    return Guarded([&] {
        if (scene == nullptr) {
            throw std::runtime_error("Bad scene handle");
        }
        srt::DeviceScene* s = FromHandle(scene);
        Bind bind(s->device());
        const srt::DeviceScene::StageTimes t = s->TakeTimes();
        if (launches != nullptr) {
            *launches = t.launches;
        }
        if (prepare_ms != nullptr) {
            *prepare_ms = t.prepare_ms;
        }
        if (bin_ms != nullptr) {
            *bin_ms = t.bin_ms;
        }
        if (trace_ms != nullptr) {
            *trace_ms = t.kernel_ms;
        }
    });
}

static_assert(SRT_SPLIT_BANDS == srt::EngineOptions::kBands && SRT_SPLIT_FRAMES == srt::EngineOptions::kFrames,
              "include/srt_render.h SRT_SPLIT_*");
static_assert(SRT_EXCHANGE_ALLTOALL == srt::EngineOptions::kAllToAll &&
                  SRT_EXCHANGE_ROTATING == srt::EngineOptions::kRotatingGather &&
                  SRT_EXCHANGE_ROOT == srt::EngineOptions::kRootGather &&
                  SRT_EXCHANGE_SHARE == srt::EngineOptions::kShare,
              "include/srt_render.h SRT_EXCHANGE_*");

}  // extern "C"

namespace {
srt::FrameEngine* FromHandle(srt_engine e) { return reinterpret_cast<srt::FrameEngine*>(e); }

srt::EngineOptions EngineOptionsFrom(const srt_engine_options* o) {
    srt::EngineOptions opt;
    if (o != nullptr) {
        if (o->struct_size != sizeof(srt_engine_options)) {
            throw std::runtime_error("srt_engine_options.struct_size is " + std::to_string(o->struct_size) + ", expected " +
                                     std::to_string(sizeof(srt_engine_options)) + " (a caller built against another "
                                     "include/srt_render.h)");
        }
        opt.variant = o->variant;
        opt.queues = o->queues == 0 ? opt.queues : o->queues;
        opt.batch = o->batch == 0 ? opt.batch : o->batch;
        if (o->rows != SRT_ROWS_INTERLEAVED && o->rows != SRT_ROWS_CONTIGUOUS && o->rows != SRT_ROWS_ROTATED) {
            throw std::runtime_error("Unknown rows mode " + std::to_string(o->rows));
        }
        opt.interleaved = o->rows == SRT_ROWS_INTERLEAVED;
        opt.rotate = o->rows == SRT_ROWS_ROTATED;
        opt.exchange = o->exchange;
        opt.split = o->split;
        opt.simulate = o->simulate != 0;
        opt.launch = o->launch;
        if ((o->flags & ~SRT_ENGINE_RCCL_SELF) != 0) {
            throw std::runtime_error("Unknown engine flags " + std::to_string(o->flags));
        }
        opt.rccl_self = (o->flags & SRT_ENGINE_RCCL_SELF) != 0;
        opt.share = o->share;
        opt.own_rows = o->own_rows;
    }
    return opt;
}

void CheckDevices(const int* devices, std::size_t count) {
    int present = 0;
    if (hipGetDeviceCount(&present) != hipSuccess || present <= 0) {
        throw std::runtime_error("HIP error: no HIP device available; the frame engine has no CPU path (ml* renders on the CPU "
                                 "with ML_VISIBLE_DEVICES=cpu)");
    }
    for (std::size_t i = 0; i < count; ++i) {
        if (devices[i] < 0 || devices[i] >= present) {
            throw std::runtime_error("HIP error: device " + std::to_string(devices[i]) + " not available (" +
                                     std::to_string(present) + " present)");
        }
    }
}
}  // namespace

extern "C" {

ML_API_ENTRY int srtEngineUniqueId(void* id128) {
    return Guarded([&] {
        if (id128 == nullptr) {
            throw std::runtime_error("Bad argument");
        }
        srt::FrameEngine::UniqueId(id128);
    });
}

ML_API_ENTRY srt_engine srtEngineCreate(const char* scene_path, const int* devices, size_t device_count, size_t width,
                                        size_t height, const srt_engine_options* options) {
    srt::FrameEngine* out = nullptr;
    Guarded([&] {
        if (scene_path == nullptr || devices == nullptr || device_count == 0) {
            throw std::runtime_error("Bad argument");
        }
        CheckDevices(devices, device_count);
        const srt::Scene scene = srt::LoadScene(scene_path);
        out = new srt::FrameEngine(scene, std::vector<int>(devices, devices + device_count), width, height,
                                   EngineOptionsFrom(options));
    });
    return reinterpret_cast<srt_engine>(out);
}

ML_API_ENTRY srt_engine srtEngineCreateRank(const char* scene_path, int device, int rank, int world,
                                            const void* unique_id128, size_t width, size_t height,
                                            const srt_engine_options* options) {
    srt::FrameEngine* out = nullptr;
    Guarded([&] {
        if (scene_path == nullptr) {
            throw std::runtime_error("Bad argument");
        }
        CheckDevices(&device, 1);
        const srt::Scene scene = srt::LoadScene(scene_path);
        out = new srt::FrameEngine(scene, device, rank, world, unique_id128, width, height, EngineOptionsFrom(options));
    });
    return reinterpret_cast<srt_engine>(out);
}

ML_API_ENTRY void srtEngineRelease(srt_engine engine) {
    srt::FrameEngine* e = FromHandle(engine);
    if (e != nullptr && e->wedged()) {
        // Deliberately leaked: a device worker never returned from the failed run and still executes
        // inside the engine (its state, communicators' control block and job); freeing any of it
        // would let that thread touch freed memory if its HIP call ever returns (after a GPU reset).
        return;
    }
    delete e;
}

ML_API_ENTRY int srtEngineSetInputs(srt_engine engine, const float* host_offsets, size_t count) {
    return Guarded([&] {
        if (engine == nullptr) {
            throw std::runtime_error("Bad engine handle");
        }
        FromHandle(engine)->SetInputs(host_offsets, count);
    });
}

ML_API_ENTRY int srtEngineRun(srt_engine engine, size_t batches) {
    return Guarded([&] {
        if (engine == nullptr) {
            throw std::runtime_error("Bad engine handle");
        }
        FromHandle(engine)->Run(batches);
    });
}

ML_API_ENTRY int srtEngineVerify(srt_engine engine, size_t* mismatches, size_t* checked) {
    return Guarded([&] {
        if (engine == nullptr) {
            throw std::runtime_error("Bad engine handle");
        }
        const std::size_t bad = FromHandle(engine)->Verify(checked);
        if (mismatches != nullptr) {
            *mismatches = bad;
        }
    });
}

ML_API_ENTRY int srtEngineReadFrame(srt_engine engine, size_t frame, float* host_rgba) {
    return Guarded([&] {
        if (engine == nullptr || host_rgba == nullptr) {
            throw std::runtime_error("Bad argument");
        }
        if (!FromHandle(engine)->ReadFrame(frame, host_rgba)) {
            throw std::runtime_error("Frame " + std::to_string(frame) + " is not resident on this process's devices");
        }
    });
}

ML_API_ENTRY int srtEngineStageTimes(srt_engine engine, size_t local, size_t launches, unsigned* launched,
                                     double* prepare_ms, double* bin_ms, double* trace_ms) {
    return Guarded([&] {
        if (engine == nullptr) {
            throw std::runtime_error("Bad engine handle");
        }
        const srt::DeviceScene::StageTimes t = FromHandle(engine)->MeasureStages(local, launches);
        if (launched != nullptr) {
            *launched = t.launches;
        }
        if (prepare_ms != nullptr) {
            *prepare_ms = t.prepare_ms;
        }
        if (bin_ms != nullptr) {
            *bin_ms = t.bin_ms;
        }
        if (trace_ms != nullptr) {
            *trace_ms = t.kernel_ms;
        }
    });
}

ML_API_ENTRY int srtEngineStageTimesBatch(srt_engine engine, size_t local, size_t launches, size_t frames,
                                          unsigned* launched, double* prepare_ms, double* bin_ms, double* trace_ms) {
    return Guarded([&] {
        if (engine == nullptr) {
            throw std::runtime_error("Bad engine handle");
        }
        const srt::DeviceScene::StageTimes t = FromHandle(engine)->MeasureStages(local, launches, frames);
        if (launched != nullptr) {
            *launched = t.launches;
        }
        if (prepare_ms != nullptr) {
            *prepare_ms = t.prepare_ms;
        }
        if (bin_ms != nullptr) {
            *bin_ms = t.bin_ms;
        }
        if (trace_ms != nullptr) {
            *trace_ms = t.kernel_ms;
        }
    });
}

ML_API_ENTRY int srtEnginePoolSelfTest(size_t workers, size_t failing, int mode, double timeout_s, double* elapsed_s,
                                       int* abort_calls, char* msg, size_t msg_size) {
    return Guarded([&] {
        if (workers == 0 || workers > 64 || failing >= workers || (mode != 1 && mode != 2) || !(timeout_s > 0)) {
            throw std::runtime_error("Bad argument");
        }
        const std::string e = srt::FrameEngine::PoolSelfTest(workers, failing, mode, timeout_s, elapsed_s, abort_calls);
        if (msg != nullptr && msg_size != 0) {
            const std::size_t n = std::min(e.size(), msg_size - 1);
            std::memcpy(msg, e.data(), n);
            msg[n] = '\0';
        }
    });
}

ML_API_ENTRY size_t srtShareAuto(size_t height, size_t devices) {
    return srt::ShareAuto(height, devices);
}

ML_API_ENTRY size_t srtRotateOwnRows(size_t height) {
    size_t rows = 0;
    (void)Guarded([&] { rows = srt::RotateOwnRows(height); });  // 0: SRT_ROTATE_OWN invalid (srtGetLastError)
    return rows;
}

ML_API_ENTRY size_t srtRotateSplitForLink(size_t height, size_t width, double link_gbs, double frame_us,
                                          double bytes_per_pixel) {
    return srt::RotateSplitForLink(height, width, link_gbs, frame_us, bytes_per_pixel);
}

ML_API_ENTRY int srtEngineSplit(srt_engine engine, size_t* own_rows, size_t* buffer_rows, double* link_gbs,
                                double* frame_us, int* source) {
    return Guarded([&] {
        if (engine == nullptr) {
            throw std::runtime_error("Bad engine handle");
        }
        const srt::FrameEngine::SplitInfo s = FromHandle(engine)->split_info();
        if (own_rows != nullptr) {
            *own_rows = s.own_rows;
        }
        if (buffer_rows != nullptr) {
            *buffer_rows = s.buffer_rows;
        }
        if (link_gbs != nullptr) {
            *link_gbs = s.link_gbs;
        }
        if (frame_us != nullptr) {
            *frame_us = s.frame_us;
        }
        if (source != nullptr) {
            *source = s.source;
        }
    });
}

ML_API_ENTRY int srtEngineInfo(srt_engine engine, size_t* devices, size_t* local_devices, size_t* band_rows,
                               size_t* buffer_rows, int* rccl, double* exchange_bytes_per_frame) {
    return Guarded([&] {
        if (engine == nullptr) {
            throw std::runtime_error("Bad engine handle");
        }
        const srt::FrameEngine* e = FromHandle(engine);
        if (devices != nullptr) {
            *devices = e->devices();
        }
        if (local_devices != nullptr) {
            *local_devices = e->local_devices();
        }
        if (band_rows != nullptr) {
            *band_rows = e->band_rows(0);
        }
        if (buffer_rows != nullptr) {
            *buffer_rows = e->buffer_rows();
        }
        if (rccl != nullptr) {
            *rccl = e->uses_rccl() ? 1 : 0;
        }
        if (exchange_bytes_per_frame != nullptr) {
            *exchange_bytes_per_frame = e->exchange_bytes_per_frame();
        }
    });
}

ML_API_ENTRY int srtEngineExchangeStats(srt_engine engine, size_t local, size_t* groups, double* ms_mean,
                                        double* bytes_sent) {
    return Guarded([&] {
        if (engine == nullptr) {
            throw std::runtime_error("Bad engine handle");
        }
        const srt::FrameEngine* e = FromHandle(engine);
        if (local >= e->local_devices()) {
            throw std::runtime_error("srtEngineExchangeStats: no local device " + std::to_string(local));
        }
        const srt::FrameEngine::ExchangeStats st = e->exchange_stats(local);
        if (groups != nullptr) {
            *groups = st.groups;
        }
        if (ms_mean != nullptr) {
            *ms_mean = st.ms_mean;
        }
        if (bytes_sent != nullptr) {
            *bytes_sent = st.bytes_sent;
        }
    });
}

namespace {
int ExchangeHost(const int* const* band_ids, size_t bands, size_t width, size_t height, int rows, int exchange,
                 size_t share, size_t batch, size_t batch_index, int* const* recv, size_t* recv_frames,
                 size_t* buffer_rows) {
    return Guarded([&] {
        if (bands == 0 || width == 0 || height == 0 || batch == 0 ||
            (rows != SRT_ROWS_INTERLEAVED && rows != SRT_ROWS_CONTIGUOUS && rows != SRT_ROWS_ROTATED) ||
            exchange < SRT_EXCHANGE_ALLTOALL || exchange > SRT_EXCHANGE_SHARE ||
            (rows == SRT_ROWS_ROTATED && exchange != SRT_EXCHANGE_ALLTOALL) ||
            (exchange == SRT_EXCHANGE_SHARE && (rows != SRT_ROWS_INTERLEAVED || bands < 2))) {
            throw std::runtime_error("Bad argument");
        }
        if (exchange == SRT_EXCHANGE_SHARE) {
            share = share == 0 ? srt::ShareAuto(height, bands) : share;
            if (share > 64 || (share & (share - 1)) != 0) {
                throw std::runtime_error("share must be a power of two, 1..64");
            }
        }
        // The engine's layout (EngineSplit: kShare splits the frame into share + P - 1 interleaved classes;
        // rotated over two devices band 0 takes the split an engine without a measured link uses,
        // RotateOwnRows -- env SRT_ROTATE_OWN, default 80 %)
        const srt::BandSplit split =
            srt::EngineSplit(height, bands, true, rows == SRT_ROWS_INTERLEAVED, rows == SRT_ROWS_ROTATED,
                             exchange == SRT_EXCHANGE_SHARE ? share : 0, 0);
        srt::ExchangePlan plan;
        plan.bands = bands;
        plan.batch = batch;
        plan.exchange = exchange;
        plan.rotate = rows == SRT_ROWS_ROTATED && bands > 1;
        if (buffer_rows != nullptr) {
            *buffer_rows = split.BufferRows();
        }
        if (recv_frames != nullptr) {
            for (size_t c = 0; c < bands; ++c) {
                recv_frames[c] = plan.FramesFor(batch_index, c);
            }
        }
        if (recv == nullptr) {
            return;
        }
        if (band_ids == nullptr) {
            throw std::runtime_error("Bad argument");
        }
        const size_t pixels = batch * split.BufferRows() * width;
        std::vector<std::vector<int>> in(bands);
        for (size_t d = 0; d < bands; ++d) {
            in[d].assign(band_ids[d], band_ids[d] + pixels);
        }
        const std::vector<std::vector<int>> out = srt::ExchangeOnHost(split, plan, width, batch_index, in);
        for (size_t c = 0; c < bands; ++c) {
            if (!out[c].empty()) {
                std::copy(out[c].begin(), out[c].end(), recv[c]);
            }
        }
    });
}
}  // namespace

ML_API_ENTRY int srtExchangeHost(const int* const* band_ids, size_t bands, size_t width, size_t height, int rows,
                                 int exchange, size_t batch, size_t batch_index, int* const* recv,
                                 size_t* recv_frames, size_t* buffer_rows) {
    if (exchange == SRT_EXCHANGE_SHARE) {  // needs its share parameter: srtExchangeHostShare
        return Guarded([] { throw std::runtime_error("Bad argument: the share exchange takes srtExchangeHostShare"); });
    }
    return ExchangeHost(band_ids, bands, width, height, rows, exchange, 0, batch, batch_index, recv, recv_frames,
                        buffer_rows);
}

ML_API_ENTRY int srtExchangeHostShare(const int* const* band_ids, size_t bands, size_t width, size_t height,
                                      size_t share, size_t batch, size_t batch_index, int* const* recv,
                                      size_t* recv_frames, size_t* buffer_rows) {
    return ExchangeHost(band_ids, bands, width, height, SRT_ROWS_INTERLEAVED, SRT_EXCHANGE_SHARE, share, batch,
                        batch_index, recv, recv_frames, buffer_rows);
}

ML_API_ENTRY int srtScreenBoxHost(const float* c, int mode, float* box) {
    return Guarded([&] {
        if (c == nullptr || box == nullptr || mode < 0 || mode > 2) {
            throw std::runtime_error("Bad argument");
        }
        if (!srt::HostScreenBox(c, mode, box)) {
            throw std::runtime_error("screen box: the float fast path does not apply");
        }
    });
}

#ifdef SRT_DIAG
// Diagnostic build only (make diag): not part of include/srt_render.h.
ML_API_ENTRY int srtDiagRead(void* host, size_t bytes) {
    return Guarded([&] { srt::HipCheck(srt::DiagRead(host, bytes), "srtDiagRead"); });
}
#endif

}  // extern "C"
