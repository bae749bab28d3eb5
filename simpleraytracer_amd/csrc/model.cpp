#include "model.h"

#include <stdexcept>

#include "dtype.h"
#include "image.h"
#include "utils.h"

namespace ML {

// model.cpp:73-139 order: params, model_path, then the file. The GPU side is created by the
// first SetInputInfo (it needs the frame size), so a model can be inspected on a host
// without a GPU; rendering there fails with the HIP error text.
Model::Model(ml_model_params const* params) {
    if (params == nullptr) {
        throw std::runtime_error("Bad parameters argument");
    }
    if (params->model_path == nullptr) {
        throw std::runtime_error("Bad model_path model parameter value");
    }
    m_scene = srt::LoadScene(params->model_path);
    // The scene's flags give the image data types (a TF graph's node dtypes in the reference).
    m_input_info.dtype = (m_scene.flags & srt::kFlagInputFloat16) != 0u ? ML_FLOAT16 : ML_FLOAT32;
    m_output_info.dtype = (m_scene.flags & srt::kFlagOutputFloat16) != 0u ? ML_FLOAT16 : ML_FLOAT32;
}

// model.cpp:141-159 (no "no session" failure here: a constructed model always has a scene).
ml_status Model::GetInfo(ml_image_info* input_info, ml_image_info* output_info) {
    if (input_info != nullptr) {
        *input_info = m_input_info;
    }
    if (output_info != nullptr) {
        *output_info = m_output_info;
    }
    return ML_OK;
}

// model.cpp:161-235 semantics and messages. Deviations (SURVEY.md section 8(b) latent bugs
// 2 and 3, fixed): a zero dimension is rejected up front instead of after committing it, and
// the new input info is committed only once the device buffers exist, so a failed call leaves
// the model unchanged and a retry with the same dims does real work.
ml_status Model::SetInputInfo(ml_image_info const* info) {
    m_error_cache.str("");
    if (info == nullptr) {
        m_error_cache << "Bad info parameter";
        return ML_FAIL;
    }
    if (static_cast<int>(m_input_info.dtype) != RawDataType(*info)) {
        m_error_cache << "Overriding data type " << static_cast<int>(m_input_info.dtype) << " with "
                      << RawDataType(*info);
        return ML_FAIL;
    }
    const bool dims_ok = ForEachDim([this, info](auto dim, char const* name) {
        if (m_input_info.*dim != 0 && info->*dim != m_input_info.*dim) {
            m_error_cache << "Overriding " << name << " dimension " << m_input_info.*dim << " with " << info->*dim;
            return false;
        }
        return true;
    });
    if (!dims_ok) {
        return ML_FAIL;
    }
    const bool specified = ForEachDim([this, info](auto dim, char const* name) {
        if (info->*dim == 0) {
            m_error_cache << "Input image " << name << " dimension is not specified";
            return false;
        }
        return true;
    });
    if (!specified) {
        return ML_FAIL;
    }
    // Sizes the kernels can index (32-bit pixel coordinates) and byte counts that fit size_t.
    size_t in_bytes = 0, out_bytes = 0;
    if (info->width > kMaxFrameSide || info->height > kMaxFrameSide ||
        !ImageBytes(info->width, info->height, info->channels, DataTypeSize(RawDataType(*info)), &in_bytes) ||
        !ImageBytes(info->width, info->height, 4, 4, &out_bytes)) {
        m_error_cache << "Input image size " << info->width << " x " << info->height << " x " << info->channels
                      << " exceeds the supported maximum (" << kMaxFrameSide << " per side)";
        return ML_FAIL;
    }
    const bool same = ForEachDim([this, info](auto dim, char const*) { return m_input_info.*dim == info->*dim; });
    if (same && ((m_renderer && m_renderer->configured()) || (m_cpu && m_cpu->configured()))) {
        return ML_OK;  // nothing changed
    }
    try {
        // The backend is chosen once, by the first call: the CPU only when selected explicitly.
        if (!m_renderer && !m_cpu) {
            if (srt::CpuBackendSelected()) {
                m_cpu = std::make_unique<srt::CpuRenderer>(m_scene);
            } else {
                m_renderer = std::make_unique<srt::Renderer>(m_scene, srt::VisibleDevices());
            }
        }
        if (m_cpu) {
            m_cpu->Configure(info->width, info->height);
        } else {
            m_renderer->Configure(info->width, info->height);
        }
    } catch (std::exception& e) {
        m_error_cache << e.what();
        return ML_FAIL;
    }
    m_input_info = *info;
    m_output_info = ml_image_info{m_output_info.dtype, info->width, info->height, 4};
    return ML_OK;
}

// model.cpp:237-294 checks and messages; plus (fix of latent bug 4) the output dtype check.
ml_status Model::Infer(ml_image input, ml_image output) {
    m_error_cache.str("");
    if (Image::FromHandle(input) == nullptr) {
        m_error_cache << "Bad input image handle";
        return ML_FAIL;
    }
    if (Image::FromHandle(output) == nullptr) {
        m_error_cache << "Bad output image handle";
        return ML_FAIL;
    }
    ml_image_info out_info{};
    Image::FromHandle(output)->GetInfo(&out_info);
    const bool dims_ok = ForEachDim([this, &out_info](auto dim, char const* name) {
        if (out_info.*dim != m_output_info.*dim) {
            m_error_cache << "Output image " << name << " dimension " << out_info.*dim << " does not match "
                          << m_output_info.*dim;
            return false;
        }
        return true;
    });
    if (!dims_ok) {
        return ML_FAIL;
    }
    if (RawDataType(out_info) != static_cast<int>(m_output_info.dtype)) {
        m_error_cache << "Output image data type " << RawDataType(out_info) << " does not match "
                      << static_cast<int>(m_output_info.dtype);
        return ML_FAIL;
    }
    return RenderToImage(*Image::FromHandle(input), *Image::FromHandle(output)) ? ML_OK : ML_FAIL;
}

// model.cpp:301-347 (InferToCache) counterpart: input checks, then render straight into the
// output image's (page-locked) buffer -- no intermediate host cache.
bool Model::RenderToImage(Image& input, Image& output) {
    m_error_cache.str("");
    const bool specified = ForEachDim([this](auto dim, char const* name) {
        if (m_input_info.*dim == 0) {
            m_error_cache << "Input image " << name << " dimension is not specified";
            return false;
        }
        return true;
    });
    if (!specified) {
        return false;
    }
    const size_t in_expected =
        m_input_info.width * m_input_info.height * m_input_info.channels * DataTypeSize(m_input_info.dtype);
    size_t in_size = 0;
    void* in_data = input.Map(&in_size);
    if (in_size != in_expected) {
        input.Unmap(in_data);
        m_error_cache << "Internal error: input size does not match: " << in_size << " vs " << in_expected;
        return false;
    }
    const size_t out_expected =
        m_output_info.width * m_output_info.height * m_output_info.channels * DataTypeSize(m_output_info.dtype);
    size_t out_size = 0;
    void* out_data = output.Map(&out_size);
    if (out_size != out_expected) {
        input.Unmap(in_data);
        output.Unmap(out_data);
        m_error_cache << "Internal error: output size does not match: " << out_size << " vs " << out_expected;
        return false;
    }
    bool ok = true;
    try {
        if (m_cpu) {
            m_cpu->Render(in_data, out_data);
        } else {
            m_renderer->Render(in_data, out_data);
        }
    } catch (std::exception& e) {
        m_error_cache << "Render error: " << e.what();
        ok = false;
    }
    input.Unmap(in_data);
    output.Unmap(out_data);
    return ok;
}

char* Model::GetError(char* buffer, size_t buffer_size) const {
    return FillBuffer(buffer, buffer_size, m_error_cache.str());
}

}  // namespace ML

extern "C" {

ML_API_ENTRY char* mlGetModelError(ml_model model, char* buffer, size_t buffer_size) {
    ML::Model* m = ML::Model::FromHandle(model);
    if (m == nullptr) {
        return ML::FillBuffer(buffer, buffer_size, "Bad model handle");
    }
    return m->GetError(buffer, buffer_size);
}

ML_API_ENTRY ml_status mlGetModelInfo(ml_model model, ml_image_info* input_info, ml_image_info* output_info) {
    ML::Model* m = ML::Model::FromHandle(model);
    return m == nullptr ? ML_FAIL : m->GetInfo(input_info, output_info);
}

ML_API_ENTRY ml_status mlSetModelInputInfo(ml_model model, ml_image_info const* info) {
    ML::Model* m = ML::Model::FromHandle(model);
    return m == nullptr ? ML_FAIL : m->SetInputInfo(info);
}

ML_API_ENTRY ml_status mlInfer(ml_model model, ml_image input, ml_image output) {
    ML::Model* m = ML::Model::FromHandle(model);
    return m == nullptr ? ML_FAIL : m->Infer(input, output);
}

ML_API_ENTRY void mlReleaseModel(ml_model model) { delete ML::Model::FromHandle(model); }

}  // extern "C"
