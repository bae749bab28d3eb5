/*
 * model_runner.h -- drop-in C ABI of libModelRunner.so, MI355X renderer edition.
 *
 * ABI-compatible with the reference header /root/reference/model_runner/model_runner.h
 * (same 14 entry points, same struct layouts, same enum values), but written as valid C
 * (the reference uses `ml_data_type` without the `enum` keyword at model_runner.h:102,
 * which a C compiler rejects).
 *
 * What the objects mean in this build:
 *   ml_model  -- a triangle scene (vertices, albedo, pinhole camera) loaded from
 *                ml_model_params.model_path (format: DESIGN.md "Scene file").
 *   input     -- per-pixel sample offsets, HWC float32, channels = 2 (sx, sy in pixels).
 *   output    -- RGBA float32 framebuffer, HWC, channels = 4: (r, g, b, float(tri_id)),
 *                tri_id = -1 for a miss.
 *   mlInfer   -- render one frame: primary rays -> brute-force closest hit -> shade.
 *
 * GPU selection: env ML_VISIBLE_DEVICES="0,1,..." (the semantics of
 * /root/reference/model_runner/ml.h:67-71 `visible_devices`); unset = device 0.
 * Row bands are rendered on each listed device and gathered to the first one with RCCL.
 * ML_VISIBLE_DEVICES=cpu (or empty) selects the CPU backend explicitly (a tile-binned CPU render of
 * the same canonical math, bit-identical ids). It is never a silent fallback:
 * with a GPU backend selected and no HIP device present, mlSetModelInputInfo / mlInfer return
 * ML_FAIL with the HIP error text in the model error cache.
 */
#ifndef SRT_MODEL_RUNNER_H
#define SRT_MODEL_RUNNER_H

#include <stddef.h>

#if defined(__GNUC__) && defined(RADEONPROML_BUILD)
#define ML_API_ENTRY __attribute__((visibility("default")))
#else
#define ML_API_ENTRY
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* model_runner.h:53-60 -- 24 bytes on LP64. Zero-initialise unused fields. */
typedef struct ml_model_params {
    char const* model_path;  /* scene file path */
    char const* input_node;  /* accepted and ignored (TF node name in the reference) */
    char const* output_node; /* accepted and ignored (TF node name in the reference) */
} ml_model_params;

typedef struct ml_context_t* ml_context; /* model_runner.h:65 */
typedef struct ml_model_t* ml_model;     /* model_runner.h:70 */
typedef struct ml_image_t* ml_image;     /* model_runner.h:75 */

#define ML_INVALID_HANDLE NULL

/* model_runner.h:82-86 */
typedef enum ml_status { ML_OK = 0, ML_FAIL = 1 } ml_status;

/* model_runner.h:91-95 */
typedef enum ml_data_type { ML_FLOAT32 = 0, ML_FLOAT16 = 1 } ml_data_type;

/* model_runner.h:100-106 -- 32 bytes, dtype at offset 0, width at offset 8. */
typedef struct ml_image_info {
    ml_data_type dtype;
    size_t width;    /* pixels, 0 = unspecified */
    size_t height;   /* pixels, 0 = unspecified */
    size_t channels; /* 0 = unspecified */
} ml_image_info;

/* Context (reference: context.cpp:59-105) */
ML_API_ENTRY ml_context mlCreateContext(void);
ML_API_ENTRY char* mlGetContextError(ml_context context, char* buffer, size_t buffer_size);
ML_API_ENTRY void mlReleaseContext(ml_context context);

/* Image (reference: image.cpp:80-113). Host memory, HWC; Map returns the buffer. */
ML_API_ENTRY ml_image mlCreateImage(ml_context context, ml_image_info const* info);
ML_API_ENTRY ml_status mlGetImageInfo(ml_image image, ml_image_info* info);
ML_API_ENTRY void* mlMapImage(ml_image image, size_t* size);
ML_API_ENTRY ml_status mlUnmapImage(ml_image image, void* data);
ML_API_ENTRY void mlReleaseImage(ml_image image);

/* Model (reference: model.cpp:352-395) */
ML_API_ENTRY ml_model mlCreateModel(ml_context context, ml_model_params const* params);
ML_API_ENTRY char* mlGetModelError(ml_model model, char* buffer, size_t buffer_size);
ML_API_ENTRY ml_status mlGetModelInfo(ml_model model, ml_image_info* input_info,
                                      ml_image_info* output_info);
ML_API_ENTRY ml_status mlSetModelInputInfo(ml_model model, ml_image_info const* info);
ML_API_ENTRY ml_status mlInfer(ml_model model, ml_image input, ml_image output);
ML_API_ENTRY void mlReleaseModel(ml_model model);

#ifdef __cplusplus
}
#endif

#endif /* SRT_MODEL_RUNNER_H */
