// Host (CPU) backend of an ml_model: BASELINE config C1 ("test_app single-triangle 256x256 CPU
// render, runs without a GPU"). Selected explicitly -- ML_VISIBLE_DEVICES=cpu (or set and empty,
// SURVEY.md section 8(b)) -- never as a silent fallback: without a HIP device and without that
// selection mlSetModelInputInfo fails with the HIP error.
//
// Same canonical arithmetic as the HIP kernels (bit for bit): edge records
// with explicit fma, the exact test E_A, E_B, E_C >= 0, det > 0, t = vol / det, lexicographic
// (t, id) minimum, headlight shading. A software rasterizer around it: each record's screen box
// (the kernels' double-precision solve) bins it to 16 x 16 pixel tiles whose ray boxes it can
// overlap, and each tile's pixels test only their tile's records (tiles whose rays leave the
// screen-box range test every record). Threads over tiles. Not the oracle (oracle/srt_oracle.c,
// test infrastructure, plain brute force); the tests compare the two.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

#include "scene.h"

namespace srt {

// A record's screen box on the host (the kernels' ComputeRecord choice): mode 0 = the float fast
// path (screen_box.h) where it applies, else the double solve; 1 = the double solve; 2 = the fast
// path only (false where it does not apply). box = (xlo, xhi, ylo, yhi).
bool HostScreenBox(const float c[9], int mode, float box[4]);

// Whether env ML_VISIBLE_DEVICES selects the CPU backend ("cpu", or set to the empty string).
bool CpuBackendSelected();

class CpuRenderer {
public:
    explicit CpuRenderer(const Scene& scene);
    void Configure(std::size_t width, std::size_t height);
    bool configured() const { return m_width != 0; }
    // host offsets (H x W x 2) -> host RGBA (H x W x 4); element types from the scene's flags
    // (float, or IEEE binary16 bit patterns).
    void Render(const void* host_offsets, void* host_rgba);
    static unsigned Threads();  // env SRT_CPU_THREADS, else OMP_NUM_THREADS, else the host's cores

private:
    const Scene& m_scene;
    bool m_in_half = false;
    bool m_out_half = false;
    std::size_t m_width = 0;
    std::size_t m_height = 0;
};

}  // namespace srt
