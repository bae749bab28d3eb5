// Host-side interface of the HIP render kernels (render.hip).
//
// Pipeline for one frame (or one row band of it), all on one HIP stream:
//   1. prepare: triangle list + frame -> per-triangle edge-function records (48 B each)
//   2. trace:   per pixel: primary ray from the sample offsets -> brute-force closest hit
//               over every triangle (LDS-tiled) -> shade -> RGBA float4 store
// The canonical arithmetic both kernels implement is specified in DESIGN.md "Canonical math"
// and restated independently by oracle/srt_oracle.c.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "scene.h"

namespace srt {

// Triangles per LDS tile; the edge buffer is padded to a multiple of this with disabled
// (all-NaN) records so the trace loop has no tail.
constexpr int kTileTriangles = 256;

// Edge record layout: 3 x float4 per triangle.
//   [0] = (c0A, cxA, cyA, c0B)   [1] = (cxB, cyB, c0C, cxC)   [2] = (cyC, vol, 0, 0)
// E_k(fx, fy) = fma(fy, cy_k, fma(fx, cx_k, c0_k)) for the three edges k = A, B, C.
constexpr int kEdgeFloat4PerTriangle = 3;

inline std::uint64_t PaddedTriangleCount(std::uint64_t n) {
    return (n + kTileTriangles - 1) / kTileTriangles * kTileTriangles;
}

// Trace kernel variants (DESIGN.md "Kernels"); selectable for A/B measurement.
enum TraceVariant : int {
    kTraceLds = 0,     // LDS-tiled triangle stream, 4 waves x 8 rows per lane (default)
    kTraceScalar = 1,  // wave-uniform scalar-cache triangle stream, no LDS, 1 wave per block
};

struct BandArgs {
    const float* offsets;  // device, row_count x width x 2 (band-local rows)
    float* rgba;           // device, row_count x width x 4
    std::size_t width;
    std::size_t height;     // full frame height (fy denominator)
    std::size_t row_begin;  // first frame row of the band
    std::size_t row_count;
};

// Launch the prepare kernel: writes PaddedTriangleCount(n) x 3 float4 into `edges`.
hipError_t LaunchPrepare(const float* d_vertices, std::uint64_t n, const Frame& frame, float* d_edges,
                         hipStream_t stream);

// Launch the trace kernel over one band.
hipError_t LaunchTrace(const float* d_edges, std::uint64_t n, const float* d_vertices, const float* d_albedo,
                       const Frame& frame, const float background[3], const BandArgs& band, int variant,
                       hipStream_t stream);

}  // namespace srt
