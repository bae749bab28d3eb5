// test_app -- command-line driver of the ml* API (renders one frame of a scene file).
//
// Counterpart of /root/reference/model_runner/test_app.cpp with the same options, messages,
// stderr log lines and exit status (255 on any error), so scripts written for the reference
// keep working:  test_app -m scene.srt -w 256 -h 256 [-i offsets.bin] [-o frame.bin]
// -i: raw H x W x 2 float32 sample offsets (stdin if omitted)
// -o: raw H x W x 4 float32 RGBA frame (stdout if omitted)
// -in / -on: accepted for compatibility (TF node names in the reference), ignored.
#include <cstdio>
#include <cstring>
#include <fstream>
#include <functional>
#include <iomanip>
#include <iostream>
#include <map>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "model_runner.h"

namespace {

// Positional "-name value" pairs; std::map keeps options in name order for the help text and
// for which missing option is reported first (test_app.cpp:19-116 behaviour).
class Options {
public:
    template <class T>
    void Add(const std::string& name, T* target, const std::string& help, bool optional = false) {
        Entry e;
        e.help = help;
        e.seen = optional;
        e.assign = [target, key = "-" + name](const std::string& text) {
            std::istringstream in(text);
            in >> *target;
            if (in.fail() && !in.eof()) {
                throw std::runtime_error("Bad parameter " + key + ": " + text);
            }
        };
        m_entries["-" + name] = std::move(e);
    }

    void Parse(int argc, char** argv) {
        for (int i = 1; i < argc; ++i) {
            const std::string arg = argv[i];
            if (arg == "-help") {
                throw std::runtime_error(Help());
            }
            const bool is_name = !arg.empty() && arg[0] == '-';
            if (is_name) {
                if (i % 2 == 0) {
                    throw std::runtime_error("Missing option value: " + std::string(argv[i - 1]));
                }
                continue;
            }
            if (i % 2 == 1) {
                throw std::runtime_error("Missing option name: " + arg + "\n" + Help());
            }
            auto it = m_entries.find(argv[i - 1]);
            if (it == m_entries.end()) {
                throw std::runtime_error("Unknown option: " + std::string(argv[i - 1]) + "\n" + Help());
            }
            it->second.assign(arg);
            it->second.seen = true;
        }
        for (const auto& kv : m_entries) {
            if (!kv.second.seen) {
                throw std::runtime_error("Missing option: " + kv.first + "\n" + Help());
            }
        }
    }

private:
    struct Entry {
        std::string help;
        bool seen = false;
        std::function<void(const std::string&)> assign;
    };

    std::string Help() const {
        std::ostringstream out;
        out << "Available options:\n";
        for (const auto& kv : m_entries) {
            out << std::setw(5) << "" << kv.first << ": " << kv.second.help << "\n";
        }
        return out.str();
    }

    std::map<std::string, Entry> m_entries;
};

std::string ContextError(ml_context ctx) {
    std::vector<char> buf(1024);
    return mlGetContextError(ctx, buf.data(), buf.size());
}

std::string ModelError(ml_model model) {
    std::vector<char> buf(1024);
    return mlGetModelError(model, buf.data(), buf.size());
}

std::string ReadAll(const std::string& path) {
    std::ostringstream data;
    if (path.empty()) {
        std::cerr << "Reading data from stdin...\n";
        if (std::freopen(nullptr, "rb", stdin) == nullptr) {
            throw std::runtime_error("Error reading stdin");
        }
        data << std::cin.rdbuf();
    } else {
        std::ifstream in(path, std::ios::binary);
        if (!in) {
            throw std::runtime_error("Error reading " + path);
        }
        std::cerr << "Reading data from file: " << path << "\n";
        data << in.rdbuf();
    }
    std::string bytes = data.str();
    std::cerr << "Input data size: " << bytes.size() << " bytes\n";
    return bytes;
}

void WriteAll(const std::string& path, const char* data, size_t size) {
    std::cerr << "Output data size: " << size << " bytes\n";
    if (path.empty()) {
        if (std::freopen(nullptr, "wb", stdout) == nullptr) {
            throw std::runtime_error("Error writing stdout");
        }
        std::cerr << "Writing result to stdout\n";
        std::cout.write(data, static_cast<std::streamsize>(size));
        std::cout.flush();
        return;
    }
    std::ofstream out(path, std::ios::binary);
    if (!out) {
        throw std::runtime_error("Error writing " + path);
    }
    std::cerr << "Writing result to file: " << path << "\n";
    out.write(data, static_cast<std::streamsize>(size));
}

// Releases the handles in reverse creation order, whatever path main() leaves by.
struct Handles {
    ml_context ctx = nullptr;
    ml_model model = nullptr;
    ml_image in = nullptr;
    ml_image out = nullptr;
    ~Handles() {
        if (out) mlReleaseImage(out);
        if (in) mlReleaseImage(in);
        if (model) mlReleaseModel(model);
        if (ctx) mlReleaseContext(ctx);
    }
};

void PrintInfo(const char* label, const ml_image_info& info) {
    std::cerr << label << info.width << " x " << info.height << " x " << info.channels << "\n";
}

int Run(int argc, char** argv) {
    std::string model_path, input_node, output_node, input_file, output_file;
    size_t width = 0, height = 0;
    Options opts;
    opts.Add("m", &model_path, "Path to scene file (model_path of mlCreateModel)");
    opts.Add("in", &input_node, "Input node name (accepted, ignored)", true);
    opts.Add("on", &output_node, "Output node name (accepted, ignored)", true);
    opts.Add("i", &input_file, "File with input data (H x W x 2 float32 sample offsets), stdin if omitted", true);
    opts.Add("o", &output_file, "File for output data (H x W x 4 float32 RGBA), stdout if omitted", true);
    opts.Add("w", &width, "Input image width");
    opts.Add("h", &height, "Input image height");
    opts.Parse(argc, argv);

    std::cerr << "Model path: " << model_path << "\n";
    Handles h;
    h.ctx = mlCreateContext();
    if (h.ctx == ML_INVALID_HANDLE) {
        throw std::runtime_error("Error creating context");
    }
    ml_model_params params = {};
    params.model_path = model_path.c_str();
    params.input_node = input_node.empty() ? nullptr : input_node.c_str();
    params.output_node = output_node.empty() ? nullptr : output_node.c_str();
    h.model = mlCreateModel(h.ctx, &params);
    if (h.model == ML_INVALID_HANDLE) {
        throw std::runtime_error(ContextError(h.ctx));
    }

    ml_image_info in_info{}, out_info{};
    if (mlGetModelInfo(h.model, &in_info, &out_info) != ML_OK) {
        throw std::runtime_error(ModelError(h.model));
    }
    PrintInfo("Input (init): ", in_info);
    PrintInfo("Output (init): ", out_info);

    in_info.width = width;
    in_info.height = height;
    if (mlSetModelInputInfo(h.model, &in_info) != ML_OK ||
        mlGetModelInfo(h.model, &in_info, &out_info) != ML_OK) {
        throw std::runtime_error(ModelError(h.model));
    }
    PrintInfo("Input: ", in_info);
    PrintInfo("Output: ", out_info);

    h.in = mlCreateImage(h.ctx, &in_info);
    if (h.in == ML_INVALID_HANDLE) {
        throw std::runtime_error(ContextError(h.ctx));
    }
    h.out = mlCreateImage(h.ctx, &out_info);
    if (h.out == ML_INVALID_HANDLE) {
        throw std::runtime_error(ContextError(h.ctx));
    }

    const std::string input = ReadAll(input_file);
    size_t in_size = 0;
    void* in_ptr = mlMapImage(h.in, &in_size);
    if (input.size() != in_size) {
        throw std::runtime_error("Bad input size: " + std::to_string(input.size()) +
                                 ", expected: " + std::to_string(in_size));
    }
    std::memcpy(in_ptr, input.data(), in_size);
    mlUnmapImage(h.in, in_ptr);

    if (mlInfer(h.model, h.in, h.out) != ML_OK) {
        throw std::runtime_error(ModelError(h.model));
    }

    size_t out_size = 0;
    void* out_ptr = mlMapImage(h.out, &out_size);
    const std::string frame(static_cast<const char*>(out_ptr), out_size);
    mlUnmapImage(h.out, out_ptr);
    WriteAll(output_file, frame.data(), frame.size());
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    try {
        return Run(argc, argv);
    } catch (std::exception& e) {
        std::cerr << e.what() << std::endl;
        return -1;
    }
}
