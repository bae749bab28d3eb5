// Element size per ml_data_type (reference: /root/reference/model_runner/dtype.h:40-53; the
// TensorFlow conversions at dtype.h:10-38 have no counterpart here).
#pragma once

#include <cstring>
#include <stdexcept>
#include <string>

#include "model_runner.h"

namespace ML {

static_assert(sizeof(ml_data_type) == sizeof(int), "ml_data_type is an int-sized C enum");

// The dtype field as the caller stored it. A C caller may store any int there; reading a value
// outside the enum's range as ml_data_type is undefined in C++ (UBSan's -fsanitize=enum caught
// exactly that for dtype 7, tools/asan_tests.sh), so the field is read as its int bytes.
inline int RawDataType(const ml_image_info& info) {
    int v = 0;
    std::memcpy(&v, &info.dtype, sizeof v);
    return v;
}

inline size_t DataTypeSize(int type) {
    if (type == ML_FLOAT32) {
        return 4;
    }
    if (type == ML_FLOAT16) {
        return 2;
    }
    throw std::runtime_error("Unsupported image data type: " + std::to_string(type));
}

}  // namespace ML
