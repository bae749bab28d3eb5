// Probe of the reference's error-buffer helper, compiled against
// /root/reference/model_runner/utils.h (make ref). Prints one line per case so
// tests/test_reference_boundary.py can record the reference behaviour this build deviates
// from on purpose (include/model_runner.h, simpleraytracer_amd/csrc/utils.h FillBuffer).
#include <cstdio>
#include <exception>
#include <string>

#include "utils.h"

static void Probe(size_t size, const std::string& msg) {
    char buf[64] = "UNTOUCHED";
    try {
        ML::FillBuffer(buf, size, msg);
        std::printf("%zu|%s|%s\n", size, msg.c_str(), buf);
    } catch (std::exception& e) {
        std::printf("%zu|%s|THROW\n", size, msg.c_str());
    }
}

int main() {
    Probe(64, "Bad model handle");
    Probe(4, "abcdef");
    Probe(64, "");
    Probe(0, "abc");
    Probe(7, "abcdef");
    return 0;
}
