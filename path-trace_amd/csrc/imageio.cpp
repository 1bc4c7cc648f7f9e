/*
 * imageio.cpp -- the output and environment-map formats of the reference:
 *   read_hdr  : Radiance RGBE reader (reference src/image.cpp:83-324),
 *               new-style RLE scanlines, 179 * 2^(e-136) scaling, alpha 1;
 *   read_png  : PngDecoder (src/png_decoder.cpp:40-128, libpng) restated on
 *               zlib: 8/16-bit RGB(A) and 1-8-bit palette images, Adam7,
 *               then Image::Image's byte / 255.0f (src/image.cpp:60-79);
 *   read_image: Image(string fileName) format dispatch by extension;
 *   write_hdr : MutableImage::writeHDR (src/image.cpp:398-481), byte-for-byte
 *               the same greedy run/literal encoder;
 *   write_bmp : the 24-bpp BI_RGB bottom-up BMP that SDL_SaveBMP wrote for the
 *               demo (src/test.cpp:1037-1059), bytes clamp(floor(256*c/count)).
 */
#include <zlib.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>

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

/* ------------------------------------------------------------------ PNG --
 * PngDecoder (reference src/png_decoder.cpp:40-128) + the /255 conversion of
 * Image::Image (src/image.cpp:60-79).  The reference drives libpng with
 * png_set_strip_16 (keep the high byte), png_set_packing, for palette images
 * png_set_palette_to_rgb (expands the palette and, libpng >= 1.2.9, tRNS to
 * alpha), and png_set_filler(0, AFTER) when the colour type has no alpha;
 * png_read_image deinterlaces Adam7.  Rows land in a w*4-byte-per-row RGBA
 * buffer.  Grayscale colour types come out as 1-2 bytes per pixel in that
 * 4-byte-per-pixel buffer (rows half written, the rest uninitialised), which
 * no decoder can reproduce, so they are rejected here. */
namespace
{

uint32_t be32(const uint8_t *p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

int paeth(int a, int b, int c)
{
    int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    if (pa <= pb && pa <= pc)
        return a;
    return pb <= pc ? b : c;
}

/* Reverses the scanline filters of one (sub)image in place: rows of 1 + rb bytes. */
void unfilter(uint8_t *data, size_t rows, size_t rb, int bpp)
{
    std::vector<uint8_t> zero(rb, 0);
    const uint8_t *prev = zero.data();
    for (size_t y = 0; y < rows; y++) {
        uint8_t *row = data + y * (rb + 1);
        const int f = row[0];
        uint8_t *x = row + 1;
        switch (f) {
        case 0:
            break;
        case 1:
            for (size_t i = bpp; i < rb; i++) x[i] = (uint8_t)(x[i] + x[i - bpp]);
            break;
        case 2:
            for (size_t i = 0; i < rb; i++) x[i] = (uint8_t)(x[i] + prev[i]);
            break;
        case 3:
            for (size_t i = 0; i < rb; i++) x[i] = (uint8_t)(x[i] + ((i >= (size_t)bpp ? x[i - bpp] : 0) + prev[i]) / 2);
            break;
        case 4:
            for (size_t i = 0; i < rb; i++)
                x[i] = (uint8_t)(x[i] + paeth(i >= (size_t)bpp ? x[i - bpp] : 0, prev[i], i >= (size_t)bpp ? prev[i - bpp] : 0));
            break;
        default:
            throw Error(PT_ERR_IO, "bad adaptive filter value");
        }
        prev = x;
    }
}

} // namespace

ImageRec read_png(const std::string &path)
{
    std::ifstream is(path, std::ios::binary);
    if (!is)
        throw Error(PT_ERR_IO, "can't open file : \"" + path + "\"");
    std::vector<uint8_t> file((std::istreambuf_iterator<char>(is)), std::istreambuf_iterator<char>());
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (file.size() < 8 || memcmp(file.data(), sig, 8) != 0)
        throw Error(PT_ERR_IO, "Not a PNG file");
    uint32_t w = 0, h = 0;
    int depth = 0, ctype = -1, interlace = 0;
    std::vector<uint8_t> plte, trns, idat;
    bool end = false;
    for (size_t p = 8; !end;) {
        if (p + 12 > file.size())
            throw Error(PT_ERR_IO, "Read Error");
        const uint32_t len = be32(&file[p]);
        if (len > 0x7fffffffu || p + 12 + (size_t)len > file.size())
            throw Error(PT_ERR_IO, "Read Error");
        const uint8_t *type = &file[p + 4], *d = &file[p + 8];
        const bool critical = !(type[0] & 0x20);
        const uint32_t crc = (uint32_t)crc32(crc32(0L, Z_NULL, 0), type, 4 + len);
        if (crc != be32(d + len)) {
            if (critical)
                throw Error(PT_ERR_IO, std::string((const char *)type, 4) + ": CRC error");
            p += 12 + (size_t)len; /* ancillary: libpng warns and discards */
            continue;
        }
        const std::string t((const char *)type, 4);
        if (t == "IHDR") {
            if (len != 13)
                throw Error(PT_ERR_IO, "Invalid IHDR chunk");
            w = be32(d), h = be32(d + 4), depth = d[8], ctype = d[9], interlace = d[12];
            if (w == 0 || h == 0 || w > 0x7fffffffu / 4 || h > 0x7fffffffu / 4 || d[10] != 0 || d[11] != 0 || interlace > 1)
                throw Error(PT_ERR_IO, "Invalid IHDR data");
        } else if (t == "PLTE") {
            plte.assign(d, d + len);
        } else if (t == "tRNS") {
            trns.assign(d, d + len);
        } else if (t == "IDAT") {
            idat.insert(idat.end(), d, d + len);
        } else if (t == "IEND") {
            end = true;
        }
        p += 12 + (size_t)len;
    }
    if (ctype < 0)
        throw Error(PT_ERR_IO, "Missing IHDR before IDAT");
    int channels;
    switch (ctype) {
    case 2: channels = 3; break;
    case 3: channels = 1; break;
    case 6: channels = 4; break;
    case 0:
    case 4: throw Error(PT_ERR_IO, "grayscale PNG: the reference decoder leaves rows partly unwritten");
    default: throw Error(PT_ERR_IO, "Invalid color type in IHDR");
    }
    const bool ok_depth = ctype == 3 ? (depth == 1 || depth == 2 || depth == 4 || depth == 8) : (depth == 8 || depth == 16);
    if (!ok_depth)
        throw Error(PT_ERR_IO, "Invalid bit depth in IHDR");
    if (ctype == 3 && (plte.empty() || plte.size() % 3 != 0))
        throw Error(PT_ERR_IO, "Missing PLTE before IDAT");
    const int bits = channels * depth, bpp = std::max(1, bits / 8);

    /* Adam7 passes (or the whole image) */
    struct Pass
    {
        int x0, y0, dx, dy;
    };
    static const Pass adam7[7] = {{0, 0, 8, 8}, {4, 0, 8, 8}, {0, 4, 4, 8}, {2, 0, 4, 4},
                                  {0, 2, 2, 4}, {1, 0, 2, 2}, {0, 1, 1, 2}};
    const Pass whole = {0, 0, 1, 1};
    const int npass = interlace ? 7 : 1;
    size_t raw_size = 0;
    for (int k = 0; k < npass; k++) {
        const Pass &ps = interlace ? adam7[k] : whole;
        const size_t pw = (w + ps.dx - 1 - ps.x0) / ps.dx, ph = (h + ps.dy - 1 - ps.y0) / ps.dy;
        if (w <= (uint32_t)ps.x0 || h <= (uint32_t)ps.y0 || pw == 0 || ph == 0)
            continue;
        raw_size += ph * (1 + (pw * bits + 7) / 8);
    }
    std::vector<uint8_t> raw(raw_size);
    {
        z_stream zs;
        memset(&zs, 0, sizeof zs);
        if (inflateInit(&zs) != Z_OK)
            throw Error(PT_ERR_IO, "zlib init failed");
        zs.next_in = idat.data();
        zs.avail_in = (uInt)idat.size();
        zs.next_out = raw.data();
        zs.avail_out = (uInt)raw.size();
        const int rc = inflate(&zs, Z_FINISH);
        const size_t got = raw.size() - zs.avail_out;
        inflateEnd(&zs);
        if ((rc != Z_STREAM_END && !(rc == Z_BUF_ERROR && zs.avail_out == 0)) || got != raw.size())
            throw Error(PT_ERR_IO, rc == Z_DATA_ERROR ? "Decompression error" : "Not enough image data");
    }
    ImageRec img;
    img.w = (int)w, img.h = (int)h;
    img.rgba.assign((size_t)4 * w * h, 0.0f);
    auto sample = [&](const uint8_t *row, size_t x, int c) -> int { /* 8-bit value after strip_16 / packing */
        if (depth == 16)
            return row[(x * channels + c) * 2];
        if (depth == 8)
            return row[x * channels + c];
        const size_t bit = x * depth;
        return (row[bit / 8] >> (8 - depth - (int)(bit % 8))) & ((1 << depth) - 1);
    };
    size_t off = 0;
    for (int k = 0; k < npass; k++) {
        const Pass &ps = interlace ? adam7[k] : whole;
        if (w <= (uint32_t)ps.x0 || h <= (uint32_t)ps.y0)
            continue;
        const size_t pw = (w + ps.dx - 1 - ps.x0) / ps.dx, ph = (h + ps.dy - 1 - ps.y0) / ps.dy;
        const size_t rb = (pw * bits + 7) / 8;
        unfilter(&raw[off], ph, rb, bpp);
        for (size_t py = 0; py < ph; py++) {
            const uint8_t *row = &raw[off + py * (rb + 1) + 1];
            const size_t y = ps.y0 + py * ps.dy;
            for (size_t px = 0; px < pw; px++) {
                const size_t x = ps.x0 + px * ps.dx;
                uint8_t out[4];
                if (ctype == 3) {
                    const int i = sample(row, px, 0);
                    if ((size_t)(3 * i + 2) < plte.size()) {
                        out[0] = plte[3 * i], out[1] = plte[3 * i + 1], out[2] = plte[3 * i + 2];
                    } else {
                        out[0] = out[1] = out[2] = 0; /* index past the palette: libpng zero-fills */
                    }
                    out[3] = trns.empty() ? 0 : ((size_t)i < trns.size() ? trns[i] : 255);
                } else {
                    for (int c = 0; c < channels; c++) out[c] = (uint8_t)sample(row, px, c);
                    if (channels == 3)
                        out[3] = 0; /* png_set_filler(0, PNG_FILLER_AFTER) */
                }
                float *o = &img.rgba[4 * (y * w + x)];
                for (int c = 0; c < 4; c++) o[c] = (int)out[c] / 255.0f;
            }
        }
        off += ph * (rb + 1);
    }
    return img;
}

ImageRec read_image(const std::string &path)
{
    const size_t dot = path.find_last_of('.');
    if (dot == std::string::npos)
        throw Error(PT_ERR_IO, "can't determine format");
    std::string fmt = path.substr(dot + 1);
    for (auto &c : fmt) c = (char)tolower((unsigned char)c);
    if (fmt == "png")
        return read_png(path);
    if (fmt == "hdr" || fmt == "pic")
        return read_hdr(path);
    throw Error(PT_ERR_IO, "invalid format"); /* src/image.cpp:327 */
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
