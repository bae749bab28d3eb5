#include "cpu_render.h"

#include "screen_box.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <stdexcept>
#include <thread>

namespace srt {
namespace {

constexpr int kTile = 16;             // pixels per tile side
constexpr float kScreenRange = 4.0f;  // render.h kScreenBoxRange: screen boxes bound |fx|, |fy| <= 4

// The kernels' expressions (render.hip Dot3 / Cross3 / ComputeRecord / ScreenBox / ShadePixel),
// restated for the host: explicit fma, no contraction (-ffp-contract=off), IEEE divide and sqrt.
inline float Dot3(float ax, float ay, float az, float bx, float by, float bz) {
    return std::fma(az, bz, std::fma(ay, by, ax * bx));
}
inline void Cross3(float ax, float ay, float az, float bx, float by, float bz, float& cx, float& cy, float& cz) {
    cx = ay * bz - az * by;
    cy = az * bx - ax * bz;
    cz = ax * by - ay * bx;
}

// Double -> float rounded toward -inf / +inf (the device's __double2float_rd / _ru).
inline float DownF(double v) {
    float f = static_cast<float>(v);
    if (static_cast<double>(f) > v) {
        f = std::nextafter(f, -std::numeric_limits<float>::infinity());
    }
    return f;
}
inline float UpF(double v) {
    float f = static_cast<float>(v);
    if (static_cast<double>(f) < v) {
        f = std::nextafter(f, std::numeric_limits<float>::infinity());
    }
    return f;
}

struct Box {
    float xlo, xhi, ylo, yhi;
};

// Every (fx, fy) with |fx|, |fy| <= 4 at which the float edge tests of c can all pass lies in
// this box (render.hip ScreenBox: the pairwise line intersections of the slack-shifted edges,
// solved in double, padded, rounded outward); unbounded when it cannot be bounded.
Box ScreenBox(const float c[9]) {
    const float inf = std::numeric_limits<float>::infinity();
    const Box unbounded{-inf, inf, -inf, inf};
    double gx[3], gy[3], k[3];
    for (int e = 0; e < 3; ++e) {
        const double c0 = c[3 * e], cx = c[3 * e + 1], cy = c[3 * e + 2];
        if (!(std::fabs(c0) < 1e30 && std::fabs(cx) < 1e30 && std::fabs(cy) < 1e30)) {
            return unbounded;
        }
        gx[e] = cx;
        gy[e] = cy;
        const double slack = (0x1p-24 * (std::fabs(c0) + kScreenRange * std::fabs(cx)) + 0x1p-120) * (1.0 + 1e-12);
        k[e] = c0 + slack;
    }
    const double dAB = gx[0] * gy[1] - gy[0] * gx[1];
    const double dBC = gx[1] * gy[2] - gy[1] * gx[2];
    const double dCA = gx[2] * gy[0] - gy[2] * gx[0];
    const bool spans = (dAB > 0 && dBC > 0 && dCA > 0) || (dAB < 0 && dBC < 0 && dCA < 0);
    if (!spans) {
        return unbounded;
    }
    double xlo = 1e300, xhi = -1e300, ylo = 1e300, yhi = -1e300;
    const double dv[3] = {dBC, dCA, dAB};
    for (int v = 0; v < 3; ++v) {
        const int i = (v + 1) % 3, j = (v + 2) % 3;
        const double inv = 1.0 / dv[v], ainv = std::fabs(inv);
        if (!(ainv < 1e300)) {
            return unbounded;
        }
        const double tx1 = -k[i] * gy[j], tx2 = k[j] * gy[i];
        const double ty1 = -gx[i] * k[j], ty2 = gx[j] * k[i];
        const double x = (tx1 + tx2) * inv, y = (ty1 + ty2) * inv;
        const double px = 1e-12 * ((std::fabs(tx1) + std::fabs(tx2)) * ainv + std::fabs(x)) + 1e-300;
        const double py = 1e-12 * ((std::fabs(ty1) + std::fabs(ty2)) * ainv + std::fabs(y)) + 1e-300;
        xlo = std::fmin(xlo, x - px);
        xhi = std::fmax(xhi, x + px);
        ylo = std::fmin(ylo, y - py);
        yhi = std::fmax(yhi, y + py);
    }
    if (!(xlo <= xhi && ylo <= yhi)) {
        return unbounded;
    }
    return Box{DownF(xlo), UpF(xhi), DownF(ylo), UpF(yhi)};
}

// One triangle's record: edge coefficients c, vol, screen box, shading normal (n, |n|).
struct Rec {
    float c[9];
    float vol;
    Box sb;
    float n[4];
};

Rec MakeRecord(const float* v, const Frame& f) {
    Rec r;
    const float qnan = std::numeric_limits<float>::quiet_NaN();
    const float inf = std::numeric_limits<float>::infinity();
    const float ax = v[0] - f.origin[0], ay = v[1] - f.origin[1], az = v[2] - f.origin[2];
    const float bx = v[3] - f.origin[0], by = v[4] - f.origin[1], bz = v[5] - f.origin[2];
    const float cx = v[6] - f.origin[0], cy = v[7] - f.origin[1], cz = v[8] - f.origin[2];
    float n[9];
    Cross3(bx, by, bz, cx, cy, cz, n[0], n[1], n[2]);
    Cross3(cx, cy, cz, ax, ay, az, n[3], n[4], n[5]);
    Cross3(ax, ay, az, bx, by, bz, n[6], n[7], n[8]);
    float vol = Dot3(ax, ay, az, n[0], n[1], n[2]);
    const bool disabled = !(std::isfinite(vol) && vol != 0.f);
    if (disabled) {
        std::fill(r.c, r.c + 9, qnan);
        r.vol = qnan;
        r.sb = Box{inf, -inf, inf, -inf};
    } else {
        if (vol < 0.f) {
            for (float& x : n) {
                x = -x;
            }
            vol = -vol;
        }
        for (int e = 0; e < 3; ++e) {
            const float nx = n[3 * e], ny = n[3 * e + 1], nz = n[3 * e + 2];
            r.c[3 * e + 0] = Dot3(nx, ny, nz, f.base[0], f.base[1], f.base[2]);
            r.c[3 * e + 1] = Dot3(nx, ny, nz, f.du[0], f.du[1], f.du[2]);
            r.c[3 * e + 2] = Dot3(nx, ny, nz, f.dv[0], f.dv[1], f.dv[2]);
        }
        r.vol = vol;
        float fb[4];
        r.sb = ScreenBoxFast(r.c, kScreenRange, fb) ? Box{fb[0], fb[1], fb[2], fb[3]} : ScreenBox(r.c);
    }
    const float e1x = v[3] - v[0], e1y = v[4] - v[1], e1z = v[5] - v[2];
    const float e2x = v[6] - v[0], e2y = v[7] - v[1], e2z = v[8] - v[2];
    Cross3(e1x, e1y, e1z, e2x, e2y, e2z, r.n[0], r.n[1], r.n[2]);
    r.n[3] = std::sqrt(Dot3(r.n[0], r.n[1], r.n[2], r.n[0], r.n[1], r.n[2]));
    return r;
}

// Runs f(i) for i in [0, n) over the backend's threads (work handed out in chunks).
template <class F>
void ParallelFor(std::size_t n, std::size_t chunk, F&& f) {
    const unsigned threads = std::max(1u, std::min<unsigned>(CpuRenderer::Threads(),
                                                             static_cast<unsigned>((n + chunk - 1) / chunk)));
    std::atomic<std::size_t> next{0};
    auto work = [&] {
        for (;;) {
            const std::size_t b = next.fetch_add(chunk);
            if (b >= n) {
                return;
            }
            for (std::size_t i = b; i < std::min(n, b + chunk); ++i) {
                f(i);
            }
        }
    };
    std::vector<std::thread> pool;
    for (unsigned t = 1; t < threads; ++t) {
        pool.emplace_back(work);
    }
    work();
    for (auto& t : pool) {
        t.join();
    }
}

}  // namespace

bool HostScreenBox(const float c[9], int mode, float box[4]) {
    if (mode != 1 && ScreenBoxFast(c, kScreenRange, box)) {
        return true;
    }
    if (mode == 2) {
        return false;
    }
    const Box b = ScreenBox(c);
    box[0] = b.xlo;
    box[1] = b.xhi;
    box[2] = b.ylo;
    box[3] = b.yhi;
    return true;
}

bool CpuBackendSelected() {
    const char* v = std::getenv("ML_VISIBLE_DEVICES");
    return v != nullptr && (*v == '\0' || std::strcmp(v, "cpu") == 0);
}

unsigned CpuRenderer::Threads() {
    for (const char* name : {"SRT_CPU_THREADS", "OMP_NUM_THREADS"}) {
        const char* v = std::getenv(name);
        if (v != nullptr && std::atoi(v) > 0) {
            return static_cast<unsigned>(std::atoi(v));
        }
    }
    const unsigned hw = std::thread::hardware_concurrency();
    return hw == 0 ? 1u : hw;
}

CpuRenderer::CpuRenderer(const Scene& scene)
    : m_scene(scene),
      m_in_half((scene.flags & kFlagInputFloat16) != 0u),
      m_out_half((scene.flags & kFlagOutputFloat16) != 0u) {}

void CpuRenderer::Configure(std::size_t width, std::size_t height) {
    if (width == 0 || height == 0) {
        throw std::runtime_error("CPU renderer: frame dimensions must be non-zero");
    }
    m_width = width;
    m_height = height;
}

void CpuRenderer::Render(const void* host_offsets, void* host_rgba) {
    if (!configured()) {
        throw std::runtime_error("Renderer used before Configure()");
    }
    const std::size_t W = m_width, H = m_height;
    const Frame f = MakeFrame(m_scene.camera, W, H);
    const float wf = static_cast<float>(W), hf = static_cast<float>(H);
    const std::size_t n = m_scene.triangle_count();
    // Records of every triangle (the kernels' record pass).
    std::vector<Rec> recs(n);
    ParallelFor(n, 1024, [&](std::size_t i) { recs[i] = MakeRecord(m_scene.vertices.data() + 9 * i, f); });
    // Ray positions (the kernels' GenerateRays) and each tile's ray box.
    std::vector<float> fx(W * H), fy(W * H);
    auto offset = [&](std::size_t i, int k) {
        if (m_in_half) {
            return static_cast<float>(static_cast<const _Float16*>(host_offsets)[2 * i + k]);
        }
        return static_cast<const float*>(host_offsets)[2 * i + k];
    };
    ParallelFor(H, 16, [&](std::size_t y) {
        for (std::size_t x = 0; x < W; ++x) {
            const std::size_t i = y * W + x;
            fx[i] = (static_cast<float>(x) + offset(i, 0)) / wf;
            fy[i] = (static_cast<float>(y) + offset(i, 1)) / hf;
        }
    });
    const std::size_t tx = (W + kTile - 1) / kTile, ty = (H + kTile - 1) / kTile, tiles = tx * ty;
    const float inf = std::numeric_limits<float>::infinity();
    std::vector<Box> tbox(tiles, Box{inf, -inf, inf, -inf});
    std::vector<char> usable(tiles, 0);
    ParallelFor(tiles, 8, [&](std::size_t t) {
        const std::size_t x0 = t % tx * kTile, y0 = t / tx * kTile;
        Box b{inf, -inf, inf, -inf};
        for (std::size_t y = y0; y < std::min(H, y0 + kTile); ++y) {
            for (std::size_t x = x0; x < std::min(W, x0 + kTile); ++x) {
                const float px = fx[y * W + x], py = fy[y * W + x];  // NaN drops out of fmin / fmax
                b = Box{std::fmin(b.xlo, px), std::fmax(b.xhi, px), std::fmin(b.ylo, py), std::fmax(b.yhi, py)};
            }
        }
        tbox[t] = b;
        usable[t] = b.xlo >= -kScreenRange && b.xhi <= kScreenRange && b.ylo >= -kScreenRange &&
                    b.yhi <= kScreenRange;
    });
    // Monotone column / row bounds of the usable tiles' boxes (suffix minimum of lo, prefix
    // maximum of hi): a record's candidate columns and rows by two binary searches each.
    std::vector<float> clo(tx, inf), chi(tx, -inf), rlo(ty, inf), rhi(ty, -inf);
    for (std::size_t t = 0; t < tiles; ++t) {
        if (usable[t] && tbox[t].xlo <= tbox[t].xhi) {
            const std::size_t c = t % tx, r = t / tx;
            clo[c] = std::min(clo[c], tbox[t].xlo);
            chi[c] = std::max(chi[c], tbox[t].xhi);
            rlo[r] = std::min(rlo[r], tbox[t].ylo);
            rhi[r] = std::max(rhi[r], tbox[t].yhi);
        }
    }
    for (std::size_t c = tx - 1; c-- > 0;) {
        clo[c] = std::min(clo[c], clo[c + 1]);
    }
    for (std::size_t c = 1; c < tx; ++c) {
        chi[c] = std::max(chi[c], chi[c - 1]);
    }
    for (std::size_t r = ty - 1; r-- > 0;) {
        rlo[r] = std::min(rlo[r], rlo[r + 1]);
    }
    for (std::size_t r = 1; r < ty; ++r) {
        rhi[r] = std::max(rhi[r], rhi[r - 1]);
    }
    // Bins: a record joins every usable tile whose box overlaps its screen box (ascending ids).
    // A pixel of a usable tile outside a record's screen box cannot pass its test (screen-box
    // guarantee), so skipping the pair is exact; tiles that are not usable test every record.
    std::vector<std::vector<std::uint32_t>> lists(tiles);
    for (std::size_t i = 0; i < n; ++i) {
        const Box& s = recs[i].sb;
        if (!(s.xlo <= s.xhi && s.ylo <= s.yhi)) {
            continue;  // disabled: never hits
        }
        const std::size_t c0 = std::lower_bound(chi.begin(), chi.end(), s.xlo) - chi.begin();
        const std::size_t c1 = std::upper_bound(clo.begin(), clo.end(), s.xhi) - clo.begin();
        const std::size_t r0 = std::lower_bound(rhi.begin(), rhi.end(), s.ylo) - rhi.begin();
        const std::size_t r1 = std::upper_bound(rlo.begin(), rlo.end(), s.yhi) - rlo.begin();
        for (std::size_t r = r0; r < r1; ++r) {
            for (std::size_t c = c0; c < c1; ++c) {
                const std::size_t t = r * tx + c;
                const Box& b = tbox[t];
                if (usable[t] && !(s.xhi < b.xlo || s.xlo > b.xhi || s.yhi < b.ylo || s.ylo > b.yhi)) {
                    lists[t].push_back(static_cast<std::uint32_t>(i));
                }
            }
        }
    }
    std::vector<std::uint32_t> all(n);
    for (std::size_t i = 0; i < n; ++i) {
        all[i] = static_cast<std::uint32_t>(i);
    }
    // Trace + shade, tile by tile.
    const float* albedo = m_scene.albedo.data();
    const float* bg = m_scene.background;
    ParallelFor(tiles, 1, [&](std::size_t t) {
        const std::vector<std::uint32_t>& cand = usable[t] ? lists[t] : all;
        const std::size_t x0 = t % tx * kTile, y0 = t / tx * kTile;
        for (std::size_t y = y0; y < std::min(H, y0 + kTile); ++y) {
            for (std::size_t x = x0; x < std::min(W, x0 + kTile); ++x) {
                const std::size_t p = y * W + x;
                const float px = fx[p], py = fy[p];
                float best = inf;
                int id = -1;
                for (const std::uint32_t k : cand) {  // ascending ids: strict < keeps the lowest on ties
                    const float* c = recs[k].c;
                    const float eA = std::fma(py, c[2], std::fma(px, c[1], c[0]));
                    const float eB = std::fma(py, c[5], std::fma(px, c[4], c[3]));
                    const float eC = std::fma(py, c[8], std::fma(px, c[7], c[6]));
                    if (eA >= 0.f && eB >= 0.f && eC >= 0.f) {
                        const float det = (eA + eB) + eC;
                        if (det > 0.f) {
                            const float tt = recs[k].vol / det;
                            if (tt < best) {
                                best = tt;
                                id = static_cast<int>(k);
                            }
                        }
                    }
                }
                float out[4];
                if (id < 0) {
                    out[0] = bg[0];
                    out[1] = bg[1];
                    out[2] = bg[2];
                    out[3] = -1.f;
                } else {
                    const float dx = std::fma(py, f.dv[0], std::fma(px, f.du[0], f.base[0]));
                    const float dy = std::fma(py, f.dv[1], std::fma(px, f.du[1], f.base[1]));
                    const float dz = std::fma(py, f.dv[2], std::fma(px, f.du[2], f.base[2]));
                    const float* nr = recs[id].n;
                    const float nd = Dot3(nr[0], nr[1], nr[2], dx, dy, dz);
                    const float dd = Dot3(dx, dy, dz, dx, dy, dz);
                    const float cosv = std::fmin(std::fabs(nd) / (nr[3] * std::sqrt(dd)), 1.f);
                    const float* a = albedo + 3 * static_cast<std::size_t>(id);
                    out[0] = a[0] * cosv;
                    out[1] = a[1] * cosv;
                    out[2] = a[2] * cosv;
                    out[3] = static_cast<float>(id);
                }
                if (m_out_half) {
                    _Float16* o = static_cast<_Float16*>(host_rgba) + 4 * p;
                    for (int k = 0; k < 4; ++k) {
                        o[k] = static_cast<_Float16>(out[k]);
                    }
                } else {
                    std::memcpy(static_cast<float*>(host_rgba) + 4 * p, out, sizeof(out));
                }
            }
        }
    });
}

}  // namespace srt
