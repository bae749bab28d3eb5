// Element size per ml_data_type (reference: /root/reference/model_runner/dtype.h:40-53; the
// TensorFlow conversions at dtype.h:10-38 have no counterpart here).
#pragma once

#include <stdexcept>
#include <string>

#include "model_runner.h"

namespace ML {

inline size_t DataTypeSize(ml_data_type type) {
    if (type == ML_FLOAT32) {
        return 4;
    }
    if (type == ML_FLOAT16) {
        return 2;
    }
    throw std::runtime_error("Unsupported image data type: " + std::to_string(static_cast<int>(type)));
}

}  // namespace ML
