// io.cpp -- PGM codec of the host mirror (gol/io.go:42-128) and the alive-cell scan of a host
// image (gol/distributor.go:153-166).  The reference moves one byte per channel operation and
// one byte per Write syscall (gol/io.go:76-81); here the body is read and written in one call.
#include <cstdio>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <sys/stat.h>

#include "gol.hpp"

namespace gol {

Image read_pgm(const std::string &path) {
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    if (!f) throw std::runtime_error("cannot open " + path);
    std::string data((size_t)f.tellg(), '\0');  // the whole file in one read (not char by char)
    f.seekg(0);
    if (!f.read(&data[0], (std::streamsize)data.size())) throw std::runtime_error("cannot read " + path);
    // strings.Fields semantics (gol/io.go:99): four whitespace-separated header fields, then
    // the body starts after exactly one whitespace byte.
    size_t pos = 0;
    auto field = [&]() {
        while (pos < data.size() && std::isspace((unsigned char)data[pos])) ++pos;
        const size_t b = pos;
        while (pos < data.size() && !std::isspace((unsigned char)data[pos])) ++pos;
        return data.substr(b, pos - b);
    };
    if (field() != "P5") throw std::runtime_error("Not a pgm file");
    Image img;
    img.width = std::stoi(field());
    img.height = std::stoi(field());
    if (std::stoi(field()) != 255) throw std::runtime_error("Incorrect maxval/bit depth");
    ++pos;  // the single whitespace byte ending the header
    const size_t n = (size_t)img.width * (size_t)img.height;
    if (data.size() < pos + n) throw std::runtime_error("truncated pgm body: " + path);
    img.pixels.assign(data.begin() + (long)pos, data.begin() + (long)(pos + n));
    return img;
}

void write_pgm(const std::string &path, const Image &img) {
    const size_t slash = path.find_last_of('/');
    if (slash != std::string::npos) ::mkdir(path.substr(0, slash).c_str(), 0777);  // os.Mkdir("out")
    std::FILE *f = std::fopen(path.c_str(), "wb");
    if (!f) throw std::runtime_error("cannot create " + path);
    // header exactly as gol/io.go:52-59: "P5\n<W> <H>\n255\n"
    std::fprintf(f, "P5\n%d %d\n255\n", img.width, img.height);
    const size_t n = std::fwrite(img.pixels.data(), 1, img.pixels.size(), f);
    std::fflush(f);
    std::fclose(f);
    if (n != img.pixels.size()) throw std::runtime_error("short write: " + path);
}

std::vector<Cell> alive_cells_of(const Image &img) {
    std::vector<Cell> out;
    for (int y = 0; y < img.height; ++y)
        for (int x = 0; x < img.width; ++x)
            if (img.pixels[(size_t)y * img.width + x] == 255) out.push_back({x, y});
    return out;
}

}  // namespace gol
