// Extension C entry points (include/srt_render.h): scene files and device-level stages.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <exception>
#include <string>
#include <vector>

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
                                     std::to_string(count) + " present); this renderer has no CPU path");
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

ML_API_ENTRY int srtGatherBandsHost(const void* const* bands, size_t band_count, size_t width, size_t height,
                                    int element_bytes, void* frame) {
    return Guarded([&] {
        if (bands == nullptr || frame == nullptr || band_count == 0 || (element_bytes != 2 && element_bytes != 4)) {
            throw std::runtime_error("Bad argument");
        }
        const srt::GatherPlan plan = srt::GatherPlan::Make(width, height, band_count, element_bytes);
        std::vector<unsigned char> gather(plan.bands * plan.BandBytes());
        srt::GatherOnHost(plan, bands, gather.data(), frame);
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

#ifdef SRT_DIAG
// Diagnostic build only (make diag): not part of include/srt_render.h.
ML_API_ENTRY int srtDiagRead(void* host, size_t bytes) {
    return Guarded([&] { srt::HipCheck(srt::DiagRead(host, bytes), "srtDiagRead"); });
}
#endif

}  // extern "C"
