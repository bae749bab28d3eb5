#include "scene.h"

#include <algorithm>
#include <array>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <stdexcept>

namespace srt {
namespace {

constexpr char kMagic[8] = {'S', 'R', 'T', 'S', 'C', 'N', '0', '1'};
constexpr std::uint32_t kVersion = 1;

// On-disk header, little-endian, 80 bytes. Followed by N*9 float vertices, N*3 float albedo.
struct FileHeader {
    char magic[8];
    std::uint32_t version;
    std::uint32_t flags;
    std::uint64_t triangles;
    float camera[10];  // eye[3] lookat[3] up[3] vfov_deg
    float background[3];
    float reserved;
};
static_assert(sizeof(FileHeader) == 80, "scene header layout");

struct FileCloser {
    void operator()(std::FILE* f) const { std::fclose(f); }
};
using File = std::unique_ptr<std::FILE, FileCloser>;

// PCG32 (XSH-RR 64/32), O'Neill's published reference algorithm.
class Pcg32 {
public:
    Pcg32(std::uint64_t seed, std::uint64_t stream) : m_inc((stream << 1u) | 1u) {
        Next();
        m_state += seed;
        Next();
    }
    std::uint32_t Next() {
        std::uint64_t old = m_state;
        m_state = old * 6364136223846793005ULL + m_inc;
        auto xorshifted = static_cast<std::uint32_t>(((old >> 18u) ^ old) >> 27u);
        auto rot = static_cast<std::uint32_t>(old >> 59u);
        return (xorshifted >> rot) | (xorshifted << ((32u - rot) & 31u));
    }
    // Uniform in [lo, hi) with 24 random bits, evaluated in double.
    double Uniform(double lo, double hi) {
        double u = static_cast<double>(Next() >> 8) * (1.0 / 16777216.0);
        return lo + (hi - lo) * u;
    }

private:
    std::uint64_t m_state = 0;
    std::uint64_t m_inc;
};

void SetCamera(Scene& s, float ex, float ey, float ez, float lx, float ly, float lz, float vfov) {
    const float cam[10] = {ex, ey, ez, lx, ly, lz, 0.f, 1.f, 0.f, vfov};
    std::memcpy(s.camera.eye, cam, 3 * sizeof(float));
    std::memcpy(s.camera.lookat, cam + 3, 3 * sizeof(float));
    std::memcpy(s.camera.up, cam + 6, 3 * sizeof(float));
    s.camera.vfov_deg = cam[9];
}

void AddTriangle(Scene& s, const float (&v)[9], float r, float g, float b) {
    s.vertices.insert(s.vertices.end(), v, v + 9);
    s.albedo.push_back(r);
    s.albedo.push_back(g);
    s.albedo.push_back(b);
}

// Axis-aligned quad p0,p1,p2,p3 (in order around the boundary) as two triangles.
void AddQuad(Scene& s, const float (&p)[12], float r, float g, float b) {
    const float t0[9] = {p[0], p[1], p[2], p[3], p[4], p[5], p[6], p[7], p[8]};
    const float t1[9] = {p[0], p[1], p[2], p[6], p[7], p[8], p[9], p[10], p[11]};
    AddTriangle(s, t0, r, g, b);
    AddTriangle(s, t1, r, g, b);
}

Scene MakeSingleTriangle() {
    Scene s;
    SetCamera(s, 0.f, 0.f, 0.f, 0.f, 0.f, 1.f, 60.f);
    s.background[0] = 0.05f;
    s.background[1] = 0.05f;
    s.background[2] = 0.08f;
    const float v[9] = {-0.5f, -0.5f, 2.f, 0.5f, -0.5f, 2.f, 0.f, 0.5f, 2.f};
    AddTriangle(s, v, 0.9f, 0.6f, 0.3f);
    return s;
}

// Unit box [0,1]^3 open towards -z: floor, ceiling, back, two side walls (10 triangles) and a
// light quad just under the ceiling (2 triangles). Camera outside the open side.
Scene MakeCornell() {
    Scene s;
    SetCamera(s, 0.5f, 0.5f, -1.4f, 0.5f, 0.5f, 0.f, 40.f);
    const float white = 0.73f;
    const float floor_q[12] = {0, 0, 0, 1, 0, 0, 1, 0, 1, 0, 0, 1};
    const float ceil_q[12] = {0, 1, 0, 0, 1, 1, 1, 1, 1, 1, 1, 0};
    const float back_q[12] = {0, 0, 1, 1, 0, 1, 1, 1, 1, 0, 1, 1};
    const float xlo_q[12] = {0, 0, 0, 0, 0, 1, 0, 1, 1, 0, 1, 0};
    const float xhi_q[12] = {1, 0, 0, 1, 1, 0, 1, 1, 1, 1, 0, 1};
    const float light_q[12] = {0.35f, 0.999f, 0.35f, 0.65f, 0.999f, 0.35f,
                               0.65f, 0.999f, 0.65f, 0.35f, 0.999f, 0.65f};
    AddQuad(s, floor_q, white, white, white);
    AddQuad(s, ceil_q, white, white, white);
    AddQuad(s, back_q, white, white, white);
    AddQuad(s, xlo_q, 0.12f, 0.45f, 0.15f);
    AddQuad(s, xhi_q, 0.65f, 0.05f, 0.05f);
    AddQuad(s, light_q, 1.f, 1.f, 1.f);
    return s;
}

// centroids uniform in [-1,1]^2 x [2,4], vertices = centroid +
// uniform[-s,s]^3, albedo uniform [0.2,1]^3, camera at the origin looking +z, vfov 60.
Scene MakeSoup(std::uint64_t n, std::uint64_t seed, float size) {
    Scene s;
    SetCamera(s, 0.f, 0.f, 0.f, 0.f, 0.f, 1.f, 60.f);
    s.background[0] = 0.02f;
    s.background[1] = 0.02f;
    s.background[2] = 0.02f;
    s.vertices.reserve(n * 9);
    s.albedo.reserve(n * 3);
    Pcg32 rng(seed, 0x5EEDu);
    const double h = size;
    for (std::uint64_t i = 0; i < n; ++i) {
        const double c[3] = {rng.Uniform(-1.0, 1.0), rng.Uniform(-1.0, 1.0), rng.Uniform(2.0, 4.0)};
        for (int v = 0; v < 3; ++v) {
            for (int k = 0; k < 3; ++k) {
                s.vertices.push_back(static_cast<float>(c[k] + rng.Uniform(-h, h)));
            }
        }
        for (int k = 0; k < 3; ++k) {
            s.albedo.push_back(static_cast<float>(rng.Uniform(0.2, 1.0)));
        }
    }
    return s;
}

[[noreturn]] void ObjError(const std::string& path, std::size_t line, const std::string& what) {
    throw std::runtime_error("Error reading scene file: " + path + ": line " + std::to_string(line) + ": " + what);
}

bool EndsWithObj(const std::string& path) {
    if (path.size() < 4) {
        return false;
    }
    std::string ext = path.substr(path.size() - 4);
    for (char& c : ext) {
        c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
    }
    return ext == ".obj";
}

// Parses `count` floats from the rest of a line; false if fewer are present or one is malformed.
bool ReadFloats(std::istringstream& in, float* out, int count) {
    for (int k = 0; k < count; ++k) {
        std::string tok;
        if (!(in >> tok)) {
            return false;
        }
        char* end = nullptr;
        out[k] = std::strtof(tok.c_str(), &end);
        if (end == tok.c_str() || *end != '\0') {
            return false;
        }
    }
    return true;
}

// Diffuse colours (Kd) of the materials of an .mtl file; a missing file yields none.
std::map<std::string, std::array<float, 3>> ReadMtl(const std::string& path) {
    std::map<std::string, std::array<float, 3>> out;
    std::ifstream f(path);
    std::string line, current;
    while (std::getline(f, line)) {
        std::istringstream in(line);
        std::string key;
        if (!(in >> key)) {
            continue;
        }
        if (key == "newmtl") {
            in >> current;
            out[current] = {0.8f, 0.8f, 0.8f};
        } else if (key == "Kd" && !current.empty()) {
            float kd[3];
            if (ReadFloats(in, kd, 3)) {
                out[current] = {kd[0], kd[1], kd[2]};
            }
        }
    }
    return out;
}

// Wavefront OBJ subset: `v x y z [w]`, `f a b c ...` with `i`, `i/t`,
// `i//n`, `i/t/n` and negative (relative) indices, polygons fan-triangulated (v0, vk, vk+1);
// `mtllib` + `usemtl` give per-face albedo from the materials' Kd (default 0.8 grey);
// every other statement (vt, vn, o, g, s, l, p, ...) is ignored. Two comment directives set
// what OBJ cannot express: `# srt camera ex ey ez lx ly lz ux uy uz vfov_deg` and
// `# srt background r g b`. Without a camera directive the camera looks along +z at the
// centre of the bounding box from where the box's bounding sphere fills a 60-degree view.
Scene LoadObj(const std::string& path) {
    std::ifstream f(path);
    if (!f) {
        throw std::runtime_error("Error reading scene file: " + path + ": cannot open");
    }
    const std::string dir = path.find('/') == std::string::npos ? "" : path.substr(0, path.rfind('/') + 1);
    std::vector<float> pos;  // 3 per vertex
    std::map<std::string, std::array<float, 3>> materials;
    std::array<float, 3> albedo = {0.8f, 0.8f, 0.8f};
    Scene s;
    bool have_camera = false;
    std::string line;
    std::size_t lineno = 0;
    while (std::getline(f, line)) {
        ++lineno;
        if (!line.empty() && line.back() == '\r') {
            line.pop_back();
        }
        std::istringstream in(line);
        std::string key;
        if (!(in >> key)) {
            continue;
        }
        if (key[0] == '#') {
            std::string tag, what;
            std::istringstream c(line.substr(line.find('#') + 1));
            if ((c >> tag >> what) && tag == "srt") {
                if (what == "camera") {
                    float cam[10];
                    if (!ReadFloats(c, cam, 10)) {
                        ObjError(path, lineno, "srt camera needs 10 numbers");
                    }
                    std::memcpy(s.camera.eye, cam, 3 * sizeof(float));
                    std::memcpy(s.camera.lookat, cam + 3, 3 * sizeof(float));
                    std::memcpy(s.camera.up, cam + 6, 3 * sizeof(float));
                    s.camera.vfov_deg = cam[9];
                    have_camera = true;
                } else if (what == "background") {
                    if (!ReadFloats(c, s.background, 3)) {
                        ObjError(path, lineno, "srt background needs 3 numbers");
                    }
                } else {
                    ObjError(path, lineno, "unknown srt directive '" + what + "'");
                }
            }
            continue;
        }
        if (key == "v") {
            float v[3];
            if (!ReadFloats(in, v, 3)) {
                ObjError(path, lineno, "vertex needs 3 coordinates");
            }
            pos.insert(pos.end(), v, v + 3);
        } else if (key == "f") {
            std::vector<std::uint64_t> idx;
            std::string tok;
            const long long nv = static_cast<long long>(pos.size() / 3);
            while (in >> tok) {
                char* end = nullptr;
                const long long i = std::strtoll(tok.c_str(), &end, 10);
                if (end == tok.c_str() || (*end != '\0' && *end != '/')) {
                    ObjError(path, lineno, "bad face index '" + tok + "'");
                }
                const long long r = i > 0 ? i - 1 : nv + i;  // 1-based, or relative when negative
                if (i == 0 || r < 0 || r >= nv) {
                    ObjError(path, lineno, "face index " + std::to_string(i) + " out of range (" +
                                               std::to_string(nv) + " vertices so far)");
                }
                idx.push_back(static_cast<std::uint64_t>(r));
            }
            if (idx.size() < 3) {
                ObjError(path, lineno, "face needs at least 3 vertices");
            }
            for (std::size_t k = 1; k + 1 < idx.size(); ++k) {
                const std::uint64_t c[3] = {idx[0], idx[k], idx[k + 1]};
                for (std::uint64_t v : c) {
                    s.vertices.insert(s.vertices.end(), pos.begin() + 3 * v, pos.begin() + 3 * v + 3);
                }
                s.albedo.insert(s.albedo.end(), albedo.begin(), albedo.end());
            }
        } else if (key == "mtllib") {
            std::string name;
            while (in >> name) {
                for (const auto& m : ReadMtl(dir + name)) {
                    materials[m.first] = m.second;
                }
            }
        } else if (key == "usemtl") {
            std::string name;
            in >> name;
            const auto it = materials.find(name);
            albedo = it != materials.end() ? it->second : std::array<float, 3>{0.8f, 0.8f, 0.8f};
        }
    }
    if (s.vertices.empty()) {
        throw std::runtime_error("Error reading scene file: " + path + ": no faces");
    }
    if (s.triangle_count() > (1ULL << 31)) {
        throw std::runtime_error("Error reading scene file: " + path + ": too many triangles");
    }
    if (!have_camera) {
        double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
        for (std::size_t i = 0; i < s.vertices.size(); i += 3) {
            for (int k = 0; k < 3; ++k) {
                if (std::isfinite(s.vertices[i + k])) {
                    lo[k] = std::fmin(lo[k], s.vertices[i + k]);
                    hi[k] = std::fmax(hi[k], s.vertices[i + k]);
                }
            }
        }
        if (!(lo[0] <= hi[0] && lo[1] <= hi[1] && lo[2] <= hi[2])) {
            throw std::runtime_error("Error reading scene file: " + path + ": no finite vertices");
        }
        const double c[3] = {(lo[0] + hi[0]) / 2, (lo[1] + hi[1]) / 2, (lo[2] + hi[2]) / 2};
        const double r = 0.5 * std::sqrt((hi[0] - lo[0]) * (hi[0] - lo[0]) + (hi[1] - lo[1]) * (hi[1] - lo[1]) +
                                         (hi[2] - lo[2]) * (hi[2] - lo[2]));
        const double dist = (r > 0.0 ? r : 1.0) / std::sin(30.0 * 3.14159265358979323846 / 180.0);
        const float cam[10] = {static_cast<float>(c[0]), static_cast<float>(c[1]), static_cast<float>(c[2] - dist),
                               static_cast<float>(c[0]), static_cast<float>(c[1]), static_cast<float>(c[2]),
                               0.f, 1.f, 0.f, 60.f};
        std::memcpy(s.camera.eye, cam, 3 * sizeof(float));
        std::memcpy(s.camera.lookat, cam + 3, 3 * sizeof(float));
        std::memcpy(s.camera.up, cam + 6, 3 * sizeof(float));
        s.camera.vfov_deg = cam[9];
    }
    if (!(s.camera.vfov_deg > 0.f && s.camera.vfov_deg < 180.f)) {
        throw std::runtime_error("Error reading scene file: " + path + ": bad camera vfov");
    }
    return s;
}

}  // namespace

Scene LoadScene(const std::string& path) {
    if (EndsWithObj(path)) {
        return LoadObj(path);
    }
    File f(std::fopen(path.c_str(), "rb"));
    if (!f) {
        throw std::runtime_error("Error reading scene file: " + path + ": cannot open");
    }
    FileHeader h{};
    if (std::fread(&h, sizeof(h), 1, f.get()) != 1) {
        throw std::runtime_error("Error reading scene file: " + path + ": truncated header");
    }
    if (std::memcmp(h.magic, kMagic, sizeof(kMagic)) != 0) {
        throw std::runtime_error("Error reading scene file: " + path + ": bad magic");
    }
    if (h.version != kVersion) {
        throw std::runtime_error("Error reading scene file: " + path + ": unsupported version " +
                                 std::to_string(h.version));
    }
    // 2^31 triangles is far beyond 288 GB of edge records; reject nonsense counts early.
    if (h.triangles == 0 || h.triangles > (1ULL << 31)) {
        throw std::runtime_error("Error reading scene file: " + path + ": bad triangle count " +
                                 std::to_string(h.triangles));
    }
    Scene s;
    std::memcpy(s.camera.eye, h.camera, 3 * sizeof(float));
    std::memcpy(s.camera.lookat, h.camera + 3, 3 * sizeof(float));
    std::memcpy(s.camera.up, h.camera + 6, 3 * sizeof(float));
    s.camera.vfov_deg = h.camera[9];
    std::memcpy(s.background, h.background, sizeof(s.background));
    s.vertices.resize(h.triangles * 9);
    s.albedo.resize(h.triangles * 3);
    if (std::fread(s.vertices.data(), sizeof(float), s.vertices.size(), f.get()) != s.vertices.size() ||
        std::fread(s.albedo.data(), sizeof(float), s.albedo.size(), f.get()) != s.albedo.size()) {
        throw std::runtime_error("Error reading scene file: " + path + ": truncated triangle data");
    }
    if (std::fgetc(f.get()) != EOF) {
        throw std::runtime_error("Error reading scene file: " + path + ": trailing bytes after the triangle data");
    }
    if ((h.flags & ~kKnownFlags) != 0u) {
        throw std::runtime_error("Error reading scene file: " + path + ": unknown flags " + std::to_string(h.flags));
    }
    s.flags = h.flags;
    if (!(s.camera.vfov_deg > 0.f && s.camera.vfov_deg < 180.f)) {
        throw std::runtime_error("Error reading scene file: " + path + ": bad camera vfov");
    }
    return s;
}

void SaveScene(const Scene& s, const std::string& path) {
    if (s.vertices.size() % 9 != 0 || s.albedo.size() != s.vertices.size() / 3) {
        throw std::runtime_error("Inconsistent scene arrays");
    }
    FileHeader h{};
    std::memcpy(h.magic, kMagic, sizeof(kMagic));
    h.version = kVersion;
    h.triangles = s.triangle_count();
    h.flags = s.flags;
    std::memcpy(h.camera, s.camera.eye, 3 * sizeof(float));
    std::memcpy(h.camera + 3, s.camera.lookat, 3 * sizeof(float));
    std::memcpy(h.camera + 6, s.camera.up, 3 * sizeof(float));
    h.camera[9] = s.camera.vfov_deg;
    std::memcpy(h.background, s.background, sizeof(h.background));
    File f(std::fopen(path.c_str(), "wb"));
    if (!f) {
        throw std::runtime_error("Error writing scene file: " + path);
    }
    if (std::fwrite(&h, sizeof(h), 1, f.get()) != 1 ||
        std::fwrite(s.vertices.data(), sizeof(float), s.vertices.size(), f.get()) != s.vertices.size() ||
        std::fwrite(s.albedo.data(), sizeof(float), s.albedo.size(), f.get()) != s.albedo.size()) {
        throw std::runtime_error("Error writing scene file: " + path);
    }
}

Scene MakeScene(int kind, std::uint64_t triangles, std::uint64_t seed, float size) {
    switch (kind) {
        case kSceneTriangle:
            return MakeSingleTriangle();
        case kSceneCornell:
            return MakeCornell();
        case kSceneSoup:
            if (triangles == 0) {
                throw std::runtime_error("Soup scene needs a positive triangle count");
            }
            return MakeSoup(triangles, seed, size > 0.f ? size : (triangles >= 1000000 ? 0.01f : 0.02f));
        default:
            throw std::runtime_error("Unknown scene kind: " + std::to_string(kind));
    }
}

Frame MakeFrame(const Camera& c, std::size_t width, std::size_t height) {
    double f[3], r[3], u[3];
    for (int k = 0; k < 3; ++k) {
        f[k] = static_cast<double>(c.lookat[k]) - static_cast<double>(c.eye[k]);
    }
    const double fl = std::sqrt(f[0] * f[0] + f[1] * f[1] + f[2] * f[2]);
    for (double& v : f) v /= fl;
    const double up[3] = {c.up[0], c.up[1], c.up[2]};
    r[0] = f[1] * up[2] - f[2] * up[1];
    r[1] = f[2] * up[0] - f[0] * up[2];
    r[2] = f[0] * up[1] - f[1] * up[0];
    const double rl = std::sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
    for (double& v : r) v /= rl;
    u[0] = r[1] * f[2] - r[2] * f[1];
    u[1] = r[2] * f[0] - r[0] * f[2];
    u[2] = r[0] * f[1] - r[1] * f[0];
    const double half_h = std::tan(static_cast<double>(c.vfov_deg) * 3.14159265358979323846 / 360.0);
    const double half_w = half_h * static_cast<double>(width) / static_cast<double>(height);
    Frame fr{};
    for (int k = 0; k < 3; ++k) {
        fr.origin[k] = c.eye[k];
        fr.base[k] = static_cast<float>(f[k] - half_w * r[k] + half_h * u[k]);
        fr.du[k] = static_cast<float>(2.0 * half_w * r[k]);
        fr.dv[k] = static_cast<float>(-2.0 * half_h * u[k]);
    }
    return fr;
}

}  // namespace srt
