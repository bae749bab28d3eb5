// ML::Image -- host-resident HWC image behind an ml_image handle.
// Reference: /root/reference/model_runner/image.{h,cpp}. Same validation order and messages;
// the buffer is page-locked (hipHostMalloc) when a HIP device is present so the framebuffer
// D2H copy of mlInfer runs at PCIe rate, and plain zeroed host memory otherwise.
#pragma once

#include <cstddef>

#include "model_runner.h"

namespace ML {

class Image {
public:
    static ml_image MakeHandle(Image* image) { return reinterpret_cast<ml_image>(image); }
    static Image* FromHandle(ml_image image) { return reinterpret_cast<Image*>(image); }

    explicit Image(ml_image_info const* info);
    ~Image();
    Image(const Image&) = delete;
    Image& operator=(const Image&) = delete;

    ml_status GetInfo(ml_image_info* info) const;
    void* Map(size_t* size);
    ml_status Unmap(void* data);

    const ml_image_info& info() const { return m_info; }
    size_t bytes() const { return m_bytes; }
    void* data() { return m_data; }

private:
    ml_image_info m_info{};
    void* m_data = nullptr;
    size_t m_bytes = 0;
    bool m_pinned = false;
};

}  // namespace ML
