#include "image.h"

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <new>
#include <stdexcept>
#include <string>

#include "dtype.h"
#include "utils.h"

namespace ML {
namespace {

bool HipDevicePresent() {
    int count = 0;
    return hipGetDeviceCount(&count) == hipSuccess && count > 0;
}

}  // namespace

// Validation order as image.cpp:22-44: null info, dtype, then width/height/channels.
Image::Image(ml_image_info const* info) {
    if (info == nullptr) {
        throw std::runtime_error("Bad image information argument");
    }
    const size_t item = DataTypeSize(RawDataType(*info));
    ForEachDim([info](auto dim, char const* name) {
        if (info->*dim == 0) {
            throw std::runtime_error(std::string("Unspecified image ") + name + " dimension");
        }
        return true;
    });
    m_info = *info;
    if (!ImageBytes(m_info.width, m_info.height, m_info.channels, item, &m_bytes)) {
        throw std::runtime_error("Image size overflows: " + std::to_string(m_info.width) + " x " +
                                 std::to_string(m_info.height) + " x " + std::to_string(m_info.channels));
    }
    if (HipDevicePresent() && hipHostMalloc(&m_data, m_bytes, hipHostMallocDefault) == hipSuccess) {
        m_pinned = true;
    } else {
        m_data = std::malloc(m_bytes);
        if (m_data == nullptr) {
            throw std::bad_alloc();
        }
    }
    std::memset(m_data, 0, m_bytes);
}

Image::~Image() {
    if (m_pinned) {
        (void)hipHostFree(m_data);
    } else {
        std::free(m_data);
    }
}

ml_status Image::GetInfo(ml_image_info* info) const {
    if (info == nullptr) {
        return ML_FAIL;
    }
    *info = m_info;
    return ML_OK;
}

void* Image::Map(size_t* size) {
    if (size != nullptr) {
        *size = m_bytes;
    }
    return m_data;
}

ml_status Image::Unmap(void* data) { return data == m_data ? ML_OK : ML_FAIL; }

}  // namespace ML

extern "C" {

ML_API_ENTRY ml_status mlGetImageInfo(ml_image image, ml_image_info* info) {
    ML::Image* img = ML::Image::FromHandle(image);
    return img == nullptr ? ML_FAIL : img->GetInfo(info);
}

ML_API_ENTRY void* mlMapImage(ml_image image, size_t* size) {
    ML::Image* img = ML::Image::FromHandle(image);
    return img == nullptr ? nullptr : img->Map(size);
}

ML_API_ENTRY ml_status mlUnmapImage(ml_image image, void* data) {
    ML::Image* img = ML::Image::FromHandle(image);
    return img == nullptr ? ML_FAIL : img->Unmap(data);
}

ML_API_ENTRY void mlReleaseImage(ml_image image) { delete ML::Image::FromHandle(image); }

}  // extern "C"
