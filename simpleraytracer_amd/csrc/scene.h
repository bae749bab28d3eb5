// Scene = what an ml_model holds in this build: a triangle list, per-triangle albedo and a
// pinhole camera ("Model = a triangle scene loaded from model_path").
// The reference Model held a TF GraphDef instead (/root/reference/model_runner/model.h:34).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace srt {

// Scene file kinds produced by the built-in generators (DESIGN.md "Scene file").
enum SceneKind : int {
    kSceneTriangle = 0,  // config C1: one triangle, 256x256
    kSceneCornell = 1,   // config C2: 12-triangle Cornell box
    kSceneSoup = 2,      // configs C3-C5: synthetic triangle soup
};

struct Camera {
    float eye[3];
    float lookat[3];
    float up[3];
    float vfov_deg;  // vertical field of view
};

// Affine primary-ray frame for one resolution: the (unnormalised) direction of the ray
// through image position (fx, fy) in [0,1]^2 (fx = column / W, fy = row / H, row 0 = top) is
//   d = base + fx * du + fy * dv.
struct Frame {
    float origin[3];
    float base[3];
    float du[3];
    float dv[3];
};

// Scene file header flags: the data types of the model's images (the role a TF graph's
// input / output node dtypes had in the reference, model.cpp:23-56).
constexpr std::uint32_t kFlagOutputFloat16 = 1u;  // output image ML_FLOAT16 (else ML_FLOAT32)
constexpr std::uint32_t kFlagInputFloat16 = 2u;   // input image ML_FLOAT16 (else ML_FLOAT32)
constexpr std::uint32_t kKnownFlags = kFlagOutputFloat16 | kFlagInputFloat16;

struct Scene {
    Camera camera{};
    std::uint32_t flags = 0;  // kFlag*
    float background[3] = {0.f, 0.f, 0.f};
    std::vector<float> vertices;  // N x 9: v0.xyz v1.xyz v2.xyz
    std::vector<float> albedo;    // N x 3: r g b

    std::uint64_t triangle_count() const { return vertices.size() / 9; }
};

// Scene file: the binary format, or Wavefront OBJ when the path ends in
// ".obj" (scene.cpp LoadObj). Throws std::runtime_error with a descriptive message on failure.
Scene LoadScene(const std::string& path);
void SaveScene(const Scene& scene, const std::string& path);

// Deterministic generators (own PCG32; no <random> distributions, whose output is
// implementation-defined). `size` is the soup half-extent s (0 = kind default).
Scene MakeScene(int kind, std::uint64_t triangles, std::uint64_t seed, float size);

// Camera -> affine frame for a W x H image. Computed in double, rounded once to float.
Frame MakeFrame(const Camera& camera, std::size_t width, std::size_t height);

}  // namespace srt
