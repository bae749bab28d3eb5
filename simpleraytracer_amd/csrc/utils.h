// Dimension visitor and error-buffer helper shared by Context/Image/Model.
#pragma once

#include <cstring>
#include <string>

#include "model_runner.h"

namespace ML {

// Visits width, height, channels -- in that order, which fixes which error message wins when
// several dimensions are wrong (reference: /root/reference/model_runner/utils.h:12-18).
template <class Visitor>
bool ForEachDim(const Visitor& visitor) {
    return visitor(&ml_image_info::width, "width") && visitor(&ml_image_info::height, "height") &&
           visitor(&ml_image_info::channels, "channels");
}

// Copies `message` into `buffer` (NUL-terminated, truncated to buffer_size - 1 characters).
// Deliberate deviation from /root/reference/model_runner/utils.h:20-28, whose version drops the
// last character of a message that fits and throws std::out_of_range across the C ABI for an
// empty message or buffer_size == 0 (SURVEY.md section 4 probes). Here an empty message gives
// "" and buffer_size == 0 leaves the buffer untouched.
inline char* FillBuffer(char* buffer, size_t buffer_size, const std::string& message) {
    if (buffer == nullptr || buffer_size == 0) {
        return buffer;
    }
    const size_t n = message.size() < buffer_size - 1 ? message.size() : buffer_size - 1;
    std::memcpy(buffer, message.data(), n);
    buffer[n] = '\0';
    return buffer;
}

// width * height * channels * item in bytes, or false when the product overflows size_t.
inline bool ImageBytes(size_t width, size_t height, size_t channels, size_t item, size_t* bytes) {
    size_t b = item;
    for (size_t f : {width, height, channels}) {
        if (f != 0 && b > static_cast<size_t>(-1) / f) {
            return false;
        }
        b *= f;
    }
    *bytes = b;
    return true;
}

// Largest frame side the render kernels index with 32-bit pixel coordinates.
constexpr size_t kMaxFrameSide = 1u << 30;

}  // namespace ML
