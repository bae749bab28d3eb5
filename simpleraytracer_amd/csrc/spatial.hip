// Spatial order of a scene's triangles, built on the GPU at scene load:
// the Morton code of each centroid's position in the scene camera's image plane, then a
// device radix sort (rocPRIM) of (code, id) pairs. The cull bins take records in this order
// (a bin block's 256 consecutive records fall in few tiles) and the BVH variant's implicit
// 8-wide tree is built over it. Only performance depends on the order: every frame is the
// lexicographic (t, id) minimum, whatever order the records are visited in.
#include <rocprim/device/device_radix_sort.hpp>

#include <cmath>
#include <stdexcept>

#include "render.h"

namespace srt {
namespace {

// Camera constants of the key (host, double; the scene file's camera).
struct KeyFrame {
    double eye[3], f[3], r[3], u[3];
    double fl, rl, ul, half_h;
    int valid;
};

// Image-plane Morton code of triangle i's centroid: 16-bit cells of the half-height-scaled
// image coordinates clamped to [-4, 4], y bit above x bit; 0xFFFFFFFF behind the eye (or a
// degenerate camera). Double arithmetic in a fixed order (-ffp-contract=off): the code is the
// same bits on any IEEE machine (tests/test_gpu_parity.py restates it in numpy).
__device__ __host__ inline unsigned MortonKey(const float* v, const KeyFrame& c) {
    double d[3];
    for (int k = 0; k < 3; ++k) {
        d[k] = (static_cast<double>(v[k]) + v[3 + k] + v[6 + k]) / 3.0 - c.eye[k];
    }
    const double z = (d[0] * c.f[0] + d[1] * c.f[1] + d[2] * c.f[2]) / c.fl;
    if (!(c.valid != 0 && z > 0.0 && isfinite(z))) {
        return 0xFFFFFFFFu;
    }
    const double sx = (d[0] * c.r[0] + d[1] * c.r[1] + d[2] * c.r[2]) / c.rl / z / c.half_h;
    const double sy = -(d[0] * c.u[0] + d[1] * c.u[1] + d[2] * c.u[2]) / c.ul / z / c.half_h;
    auto cell = [](double w) {
        const double q = (fmin(fmax(w, -4.0), 4.0) + 4.0) / 8.0 * 65535.0;
        return static_cast<unsigned>(isfinite(q) ? q : 0.0);
    };
    const unsigned qx = cell(sx), qy = cell(sy);
    unsigned key = 0;
    for (int b = 15; b >= 0; --b) {
        key = (key << 2) | (((qy >> b) & 1u) << 1) | ((qx >> b) & 1u);
    }
    return key;
}

__global__ __launch_bounds__(256) void MortonKeysKernel(const float* __restrict__ vertices, unsigned n, KeyFrame c,
                                                        unsigned* __restrict__ keys, unsigned* __restrict__ ids) {
    const unsigned i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) {
        keys[i] = MortonKey(vertices + 9ull * i, c);
        ids[i] = i;
    }
}

// rank[order[i]] = i; svertices[i] = (vertices[order[i]], order[i] bits, 0, 0) (render.h kSpatialStride:
// the bin kernel's record pass and the trace read a record's inputs by spatial position, three 16-B
// loads: coalesced, and no order -> vertex load chain per frame).
__global__ __launch_bounds__(256) void RankKernel(const unsigned* __restrict__ order, unsigned n,
                                                  const float* __restrict__ vertices, unsigned* __restrict__ rank,
                                                  float* __restrict__ svertices) {
    const unsigned i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) {
        const unsigned id = order[i];
        rank[id] = i;
        float* sv = svertices + static_cast<unsigned long long>(kSpatialStride) * i;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            sv[k] = vertices[9ull * id + k];
        }
        sv[9] = __uint_as_float(id);
        sv[10] = 0.f;
        sv[11] = 0.f;
    }
}

KeyFrame MakeKeyFrame(const Camera& c) {
    KeyFrame k{};
    for (int a = 0; a < 3; ++a) {
        k.eye[a] = c.eye[a];
        k.f[a] = static_cast<double>(c.lookat[a]) - static_cast<double>(c.eye[a]);
    }
    const double up[3] = {c.up[0], c.up[1], c.up[2]};
    k.r[0] = k.f[1] * up[2] - k.f[2] * up[1];
    k.r[1] = k.f[2] * up[0] - k.f[0] * up[2];
    k.r[2] = k.f[0] * up[1] - k.f[1] * up[0];
    k.u[0] = k.r[1] * k.f[2] - k.r[2] * k.f[1];
    k.u[1] = k.r[2] * k.f[0] - k.r[0] * k.f[2];
    k.u[2] = k.r[0] * k.f[1] - k.r[1] * k.f[0];
    k.fl = std::sqrt(k.f[0] * k.f[0] + k.f[1] * k.f[1] + k.f[2] * k.f[2]);
    k.rl = std::sqrt(k.r[0] * k.r[0] + k.r[1] * k.r[1] + k.r[2] * k.r[2]);
    k.ul = std::sqrt(k.u[0] * k.u[0] + k.u[1] * k.u[1] + k.u[2] * k.u[2]);
    k.half_h = std::tan(static_cast<double>(c.vfov_deg) * 3.14159265358979323846 / 360.0);
    k.valid = k.half_h > 0.0 && k.fl > 0.0 && k.rl > 0.0 && k.ul > 0.0 ? 1 : 0;
    return k;
}

void Check(hipError_t e, const char* what) {
    if (e != hipSuccess) {
        throw std::runtime_error(std::string("HIP error: ") + what + ": " + hipGetErrorString(e));
    }
}

}  // namespace

void BuildSpatialOrder(const float* d_vertices, std::uint64_t n, const Camera& camera, unsigned* d_order,
                       unsigned* d_rank, float* d_svertices, hipStream_t stream, hipEvent_t ev_begin,
                       hipEvent_t ev_end) {
    if (n == 0) {
        return;
    }
    const unsigned un = static_cast<unsigned>(n);
    unsigned *keys = nullptr, *keys_sorted = nullptr, *ids = nullptr;
    void* temp = nullptr;
    std::size_t temp_bytes = 0;
    auto release = [&] {
        (void)hipFree(keys);
        (void)hipFree(keys_sorted);
        (void)hipFree(ids);
        (void)hipFree(temp);
    };
    try {
        Check(hipMalloc(&keys, n * 4), "hipMalloc(morton keys)");
        Check(hipMalloc(&keys_sorted, n * 4), "hipMalloc(sorted keys)");
        Check(hipMalloc(&ids, n * 4), "hipMalloc(ids)");
        Check(rocprim::radix_sort_pairs(nullptr, temp_bytes, keys, keys_sorted, ids, d_order, un, 0, 32, stream),
              "rocprim::radix_sort_pairs (size query)");
        Check(hipMalloc(&temp, temp_bytes), "hipMalloc(sort temporary)");
        if (ev_begin != nullptr) {
            Check(hipEventRecord(ev_begin, stream), "hipEventRecord(order build)");
        }
        const unsigned blocks = (un + 255) / 256;
        hipLaunchKernelGGL(MortonKeysKernel, dim3(blocks), dim3(256), 0, stream, d_vertices, un, MakeKeyFrame(camera),
                           keys, ids);
        Check(hipGetLastError(), "MortonKeysKernel launch");
        // stable LSD radix sort: equal codes keep id order, so the order is unique
        Check(rocprim::radix_sort_pairs(temp, temp_bytes, keys, keys_sorted, ids, d_order, un, 0, 32, stream),
              "rocprim::radix_sort_pairs");
        hipLaunchKernelGGL(RankKernel, dim3(blocks), dim3(256), 0, stream, d_order, un, d_vertices, d_rank,
                           d_svertices);
        Check(hipGetLastError(), "RankKernel launch");
        if (ev_end != nullptr) {
            Check(hipEventRecord(ev_end, stream), "hipEventRecord(order build)");
        }
        Check(hipStreamSynchronize(stream), "spatial order build");
    } catch (...) {
        (void)hipStreamSynchronize(stream);
        release();
        throw;
    }
    release();
}

}  // namespace srt
