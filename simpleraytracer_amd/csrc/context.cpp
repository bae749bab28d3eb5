// ML::Context and its C entry points. Reference: /root/reference/model_runner/context.{h,cpp}.
// A context does not own the images/models it creates (same as the reference): they may
// outlive it. Constructor exceptions become ML_INVALID_HANDLE plus a cached message.
#include <sstream>
#include <string>

#include "image.h"
#include "model.h"
#include "model_runner.h"
#include "utils.h"

namespace ML {

class Context {
public:
    static ml_context MakeHandle(Context* c) { return reinterpret_cast<ml_context>(c); }
    static Context* FromHandle(ml_context c) { return reinterpret_cast<Context*>(c); }

    ml_image CreateImage(ml_image_info const* info) {
        m_error_cache.str("");
        try {
            return Image::MakeHandle(new Image(info));
        } catch (std::exception& e) {
            m_error_cache << e.what();
            return ML_INVALID_HANDLE;
        }
    }

    ml_model CreateModel(ml_model_params const* params) {
        m_error_cache.str("");
        try {
            return Model::MakeHandle(new Model(params));
        } catch (std::exception& e) {
            m_error_cache << e.what();
            return ML_INVALID_HANDLE;
        }
    }

    char* GetError(char* buffer, size_t buffer_size) const {
        return FillBuffer(buffer, buffer_size, m_error_cache.str());
    }

private:
    std::ostringstream m_error_cache;
};

}  // namespace ML

extern "C" {

ML_API_ENTRY ml_context mlCreateContext(void) {
    try {
        return ML::Context::MakeHandle(new ML::Context);
    } catch (...) {
        return ML_INVALID_HANDLE;
    }
}

ML_API_ENTRY char* mlGetContextError(ml_context context, char* buffer, size_t buffer_size) {
    ML::Context* c = ML::Context::FromHandle(context);
    if (c == nullptr) {
        return ML::FillBuffer(buffer, buffer_size, "Bad context handle");
    }
    return c->GetError(buffer, buffer_size);
}

ML_API_ENTRY ml_image mlCreateImage(ml_context context, ml_image_info const* info) {
    ML::Context* c = ML::Context::FromHandle(context);
    return c == nullptr ? ML_INVALID_HANDLE : c->CreateImage(info);
}

ML_API_ENTRY ml_model mlCreateModel(ml_context context, ml_model_params const* params) {
    ML::Context* c = ML::Context::FromHandle(context);
    return c == nullptr ? ML_INVALID_HANDLE : c->CreateModel(params);
}

ML_API_ENTRY void mlReleaseContext(ml_context context) { delete ML::Context::FromHandle(context); }

}  // extern "C"
