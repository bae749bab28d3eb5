// ML::Model -- a triangle scene plus its renderer (GPU, or the explicitly selected CPU backend)
// behind an ml_model handle.
// Reference: /root/reference/model_runner/model.{h,cpp} (TF GraphDef + Session there).
#pragma once

#include <memory>
#include <sstream>
#include <string>

#include "cpu_render.h"
#include "model_runner.h"
#include "renderer.h"
#include "scene.h"

namespace ML {

class Image;

class Model {
public:
    static ml_model MakeHandle(Model* model) { return reinterpret_cast<ml_model>(model); }
    static Model* FromHandle(ml_model model) { return reinterpret_cast<Model*>(model); }

    explicit Model(ml_model_params const* params);

    ml_status GetInfo(ml_image_info* input_info, ml_image_info* output_info);
    ml_status SetInputInfo(ml_image_info const* info);
    ml_status Infer(ml_image input, ml_image output);
    char* GetError(char* buffer, size_t buffer_size) const;

    const srt::Scene& scene() const { return m_scene; }

private:
    bool RenderToImage(Image& input, Image& output);

    srt::Scene m_scene;
    // Input: per-pixel sample offsets (2 channels); output: RGBA framebuffer (4 channels).
    ml_image_info m_input_info{ML_FLOAT32, 0, 0, 2};
    ml_image_info m_output_info{ML_FLOAT32, 0, 0, 4};
    std::unique_ptr<srt::Renderer> m_renderer;  // HIP devices (ML_VISIBLE_DEVICES list; unset = device 0)
    std::unique_ptr<srt::CpuRenderer> m_cpu;    // ML_VISIBLE_DEVICES=cpu (config C1 without a GPU)
    std::ostringstream m_error_cache;
};

}  // namespace ML
