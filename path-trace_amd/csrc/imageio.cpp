/*
 * imageio.cpp -- the output and environment-map formats of the reference:
 *   read_hdr  : Radiance RGBE reader (reference src/image.cpp:83-324),
 *               new-style RLE scanlines, 179 * 2^(e-136) scaling, alpha 1;
 *   write_hdr : MutableImage::writeHDR (src/image.cpp:398-481), byte-for-byte
 *               the same greedy run/literal encoder;
 *   write_bmp : the 24-bpp BI_RGB bottom-up BMP that SDL_SaveBMP wrote for the
 *               demo (src/test.cpp:1037-1059), bytes clamp(floor(256*c/count)).
 */
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>

#include "internal.h"

namespace pt
{

namespace
{

struct Reader
{
    std::ifstream is;
    int get()
    {
        char c;
        if (!is.get(c))
            throw Error(PT_ERR_IO, "unexpected EOF");
        return (unsigned char)c;
    }
    bool match(const char *s)
    {
        for (; *s; s++) {
            char c;
            if (!is.get(c) || c != *s)
                return false;
        }
        return true;
    }
};

} // namespace

ImageRec read_hdr(const std::string &path)
{
    Reader r;
    r.is.open(path, std::ios::binary);
    if (!r.is)
        throw Error(PT_ERR_IO, "can't open " + path);
    if (!r.match("#?RADIANCE\n"))
        throw Error(PT_ERR_IO, "magic string doesn't match");
    bool got_format = false;
    float scale[3] = {1, 1, 1};
    int ch = 0;
    /* header: KEY=value lines, '#' comments, blank line, then "-Y h +X w" */
    for (;;) {
        std::string key;
        bool size_line = false;
        for (;;) {
            ch = r.get();
            if (ch == '=')
                break;
            if (ch == '#') {
                while (r.get() != '\n') {
                }
                ch = '\n'; /* the reference re-examines the newline it consumed */
            }
            if (ch == ' ')
                continue;
            if (ch == '\n') {
                if (!key.empty())
                    throw Error(PT_ERR_IO, "unexpected token");
                continue;
            }
            if (ch == '+' || ch == '-') {
                if (!key.empty())
                    throw Error(PT_ERR_IO, "unexpected token");
                size_line = true;
                break;
            }
            if (!isalpha(ch))
                throw Error(PT_ERR_IO, "unexpected character");
            key += (char)ch;
        }
        if (size_line)
            break;
        if (key == "FORMAT") {
            if (got_format)
                throw Error(PT_ERR_IO, "format already specified");
            got_format = true;
            if (!r.match("32-bit_rle_rgbe\n"))
                throw Error(PT_ERR_IO, "invalid format specifier");
        } else if (key == "EXPOSURE" || key == "COLORCORR") {
            float v[3];
            int n = key == "EXPOSURE" ? 1 : 3;
            for (int k = 0; k < n; k++)
                if (!(r.is >> v[k]))
                    throw Error(PT_ERR_IO, "can't read header value");
            for (;;) {
                int c = r.get();
                if (c == '\n')
                    break;
                if (!isspace(c))
                    throw Error(PT_ERR_IO, "unexpected character");
            }
            for (int k = 0; k < 3; k++) scale[k] /= v[n == 1 ? 0 : k];
        } else {
            while (r.get() != '\n') {
            }
        }
    }
    if (ch != '-' || !r.match("Y"))
        throw Error(PT_ERR_IO, "invalid resolution string");
    int w = 0, h = 0;
    if (!(r.is >> h) || h <= 0)
        throw Error(PT_ERR_IO, "invalid resolution string");
    do {
        ch = r.get();
    } while (ch == ' ' || ch == '\t');
    if (ch != '+' || !r.match("X"))
        throw Error(PT_ERR_IO, "invalid resolution string");
    if (!(r.is >> w) || w <= 0 || w >= (1 << 15))
        throw Error(PT_ERR_IO, "invalid resolution string");
    for (;;) {
        int c = r.get();
        if (c == '\n')
            break;
        if (!isspace(c))
            throw Error(PT_ERR_IO, "unexpected character");
    }
    std::vector<uint8_t> rgbe((size_t)4 * w * h);
    for (int y = 0; y < h; y++) {
        uint8_t *line = &rgbe[(size_t)4 * w * y];
        for (int k = 0; k < 4; k++) line[k] = (uint8_t)r.get();
        if (line[0] != 2 || line[1] != 2 || (line[2] & 0x80))
            throw Error(PT_ERR_IO, "unsupported flat/old-style RLE scanline");
        if ((line[2] << 8) + line[3] != w)
            throw Error(PT_ERR_IO, "invalid line length in new compressed line");
        for (int c = 0; c < 4; c++) {
            for (int x = 0; x < w;) {
                int b = r.get();
                if (b > 0x80) {
                    int count = b - 0x80, v = r.get();
                    for (int i = 0; i < count; i++) {
                        if (x >= w)
                            throw Error(PT_ERR_IO, "line too long");
                        line[c + 4 * x++] = (uint8_t)v;
                    }
                } else {
                    for (int i = 0; i < b; i++) {
                        if (x >= w)
                            throw Error(PT_ERR_IO, "line too long");
                        line[c + 4 * x++] = (uint8_t)r.get();
                    }
                }
            }
        }
    }
    ImageRec img;
    img.w = w, img.h = h;
    img.rgba.resize((size_t)4 * w * h);
    for (size_t i = 0; i < (size_t)4 * w * h; i += 4) {
        int e = rgbe[i + 3] - 128;
        float factor = 179.0f * (float)std::pow(2.0, (double)(e - 8)); /* std::pow(float, int) -> double */
        img.rgba[i + 0] = rgbe[i + 0] * factor * scale[0];
        img.rgba[i + 1] = rgbe[i + 1] * factor * scale[1];
        img.rgba[i + 2] = rgbe[i + 2] * factor * scale[2];
        img.rgba[i + 3] = 1;
    }
    return img;
}

void write_hdr(const std::string &path, const float *rgb, int w, int h)
{
    std::ofstream os(path, std::ios::binary);
    if (!os)
        throw Error(PT_ERR_IO, "can't open file for writing");
    os << "#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n-Y " << h << " +X " << w << "\n";
    std::vector<uint8_t> line((size_t)4 * w);
    const uint8_t code[4] = {2, 2, (uint8_t)(w >> 8), (uint8_t)(w & 0xFF)};
    for (int y = 0; y < h; y++) {
        os.write((const char *)code, 4);
        for (int x = 0; x < w; x++) {
            const float *c = rgb + 3 * ((size_t)y * w + x);
            float hi = c[1] < c[2] ? c[2] : c[1];  /* std::max(g, b) */
            hi = c[0] < hi ? hi : c[0];            /* std::max(r, .) */
            float maxv = hi / 179.0f;
            uint8_t *p = &line[4 * x];
            if ((double)maxv < 1e-30) {
                p[0] = p[1] = p[2] = p[3] = 0;
                continue;
            }
            /* logf(maxV) / log(2.0) + 1e-5 in double, ceil; scale = 0.5^(lg-8)/179 */
            int lg = (int)std::ceil((double)std::log(maxv) / std::log(2.0) + 1e-5);
            float scale = (float)(std::pow(0.5, (double)(lg - 8)) / 179.0f);
            for (int k = 0; k < 3; k++) {
                int v = (int)std::floor(c[k] * scale);
                p[k] = (uint8_t)(v < 0 ? 0 : v > 0xFF ? 0xFF : v);
            }
            p[3] = (uint8_t)(lg + 128);
        }
        /* per channel: greedy literal/run encoder of the reference writer */
        for (int ch = 0; ch < 4; ch++) {
            size_t run = 0, skip = 0;
            auto at = [&](size_t x) { return line[ch + 4 * x]; };
            for (size_t x = 0; x < (size_t)w;) {
                while (run < 0x7F && skip <= 0x80 && run + skip + x < (size_t)w) {
                    while (run < 0x7F && run + skip + x < (size_t)w && at(x + skip) == at(x + skip + run)) run++;
                    if (run < 3) {
                        skip += run;
                        run = 0;
                    } else {
                        break;
                    }
                }
                if (run == 0 && skip > 0x80)
                    skip = 0x80;
                if (skip > 0) {
                    os.put((char)(uint8_t)skip);
                    for (size_t i = 0; i < skip; i++) os.put((char)at(x + i));
                    x += skip;
                    skip = 0;
                }
                if (run > 0) {
                    os.put((char)(uint8_t)(run + 0x80));
                    os.put((char)at(x));
                    x += run;
                    run = 0;
                }
            }
        }
    }
    if (!os)
        throw Error(PT_ERR_IO, "can't write to file");
}

void write_bmp(const std::string &path, const float *rgb, int w, int h, int count)
{
    int row = (3 * w + 3) & ~3;
    uint32_t img = (uint32_t)row * h, size = 54 + img;
    uint8_t hdr[54] = {'B', 'M'};
    auto u32 = [&](int off, uint32_t v) { memcpy(hdr + off, &v, 4); };
    auto u16 = [&](int off, uint16_t v) { memcpy(hdr + off, &v, 2); };
    u32(2, size);
    u32(10, 54);
    u32(14, 40);
    u32(18, (uint32_t)w);
    u32(22, (uint32_t)h);
    u16(26, 1);
    u16(28, 24);
    u32(30, 0);
    u32(34, img);
    std::ofstream os(path, std::ios::binary);
    if (!os)
        throw Error(PT_ERR_IO, "can't open file for writing");
    os.write((const char *)hdr, 54);
    std::vector<uint8_t> buf(row, 0);
    float fc = (float)count;
    for (int y = h - 1; y >= 0; y--) {
        for (int x = 0; x < w; x++) {
            const float *c = rgb + 3 * ((size_t)y * w + x);
            for (int k = 0; k < 3; k++) {
                /* max(0, min(0xFF, (int)floor(0x100 * c / count))), test.cpp:1037-1039 */
                int v = (int)std::floor(256.0f * c[k] / fc);
                v = v > 0xFF ? 0xFF : v;
                v = v < 0 ? 0 : v;
                buf[3 * x + (2 - k)] = (uint8_t)v; /* BGR */
            }
        }
        os.write((const char *)buf.data(), row);
    }
    if (!os)
        throw Error(PT_ERR_IO, "can't write to file");
}

} // namespace pt
