// vxpt -- host image I/O behind the C ABI: the offline frame writer and the
// canonical-image gate of the reference's offline driver.
//
//   vxpt_write_png_rgba32f  OfflineBackend::writeFrameBufferToPNG (OfflineBackend.cpp:191-221):
//                           clamp to [0,1], x255 truncated, rows flipped, 8-bit RGB
//   vxpt_read_png           the loader ImageData::loadFromFile uses (stb_image in the reference)
//   vxpt_image_diff         ImageDiff::compare (renderer/util/ImageDiff.cpp:94-124, 187-373)
//   vxpt_image_diff_png     ImageDiff::generateDiffImage (ImageDiff.cpp:126-185)
//
// PNG is written and read with zlib (8-bit grey / grey+alpha / RGB / RGBA /
// palette, non-interlaced); no other image library is involved.
#include <zlib.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/vxpt.h"

namespace {

struct Image {
    int w = 0, h = 0, ch = 0;
    std::vector<uint8_t> px;
};

void put32(std::vector<uint8_t> &v, uint32_t x) {
    v.push_back((uint8_t)(x >> 24)); v.push_back((uint8_t)(x >> 16));
    v.push_back((uint8_t)(x >> 8)); v.push_back((uint8_t)x);
}
uint32_t get32(const uint8_t *p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

void chunk(std::vector<uint8_t> &out, const char *type, const std::vector<uint8_t> &data) {
    put32(out, (uint32_t)data.size());
    std::vector<uint8_t> td(type, type + 4);
    td.insert(td.end(), data.begin(), data.end());
    out.insert(out.end(), td.begin(), td.end());
    put32(out, (uint32_t)crc32(0L, td.data(), (uInt)td.size()));
}

bool write_png(const std::string &path, const Image &im) {
    const int colorType = im.ch == 1 ? 0 : (im.ch == 2 ? 4 : (im.ch == 3 ? 2 : 6));
    std::vector<uint8_t> raw;
    raw.reserve((size_t)im.h * (1 + (size_t)im.w * im.ch));
    for (int y = 0; y < im.h; ++y) {
        raw.push_back(0);  // filter: none
        const uint8_t *row = im.px.data() + (size_t)y * im.w * im.ch;
        raw.insert(raw.end(), row, row + (size_t)im.w * im.ch);
    }
    uLongf zlen = compressBound((uLong)raw.size());
    std::vector<uint8_t> z(zlen);
    if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 6) != Z_OK) return false;
    z.resize(zlen);
    std::vector<uint8_t> out = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
    std::vector<uint8_t> ihdr;
    put32(ihdr, (uint32_t)im.w);
    put32(ihdr, (uint32_t)im.h);
    ihdr.push_back(8);
    ihdr.push_back((uint8_t)colorType);
    ihdr.push_back(0); ihdr.push_back(0); ihdr.push_back(0);
    chunk(out, "IHDR", ihdr);
    chunk(out, "IDAT", z);
    chunk(out, "IEND", {});
    FILE *f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    const bool ok = std::fwrite(out.data(), 1, out.size(), f) == out.size();
    std::fclose(f);
    return ok;
}

int paeth(int a, int b, int c) {
    const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    return (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
}

bool read_png(const std::string &path, Image &im) {
    FILE *f = std::fopen(path.c_str(), "rb");
    if (!f) return false;
    std::vector<uint8_t> d;
    uint8_t buf[65536];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) d.insert(d.end(), buf, buf + n);
    std::fclose(f);
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
    if (d.size() < 8 || std::memcmp(d.data(), sig, 8) != 0) return false;
    int w = 0, h = 0, depth = 0, ct = -1, interlace = 0;
    std::vector<uint8_t> idat, plte;
    for (size_t p = 8; p + 12 <= d.size();) {
        const uint32_t len = get32(&d[p]);
        if (p + 12 + len > d.size()) return false;
        const std::string type(reinterpret_cast<const char *>(&d[p + 4]), 4);
        const uint8_t *data = &d[p + 8];
        if (type == "IHDR") {
            w = (int)get32(data); h = (int)get32(data + 4);
            depth = data[8]; ct = data[9]; interlace = data[12];
        } else if (type == "PLTE") {
            plte.assign(data, data + len);
        } else if (type == "IDAT") {
            idat.insert(idat.end(), data, data + len);
        } else if (type == "IEND") {
            break;
        }
        p += 12 + len;
    }
    if (w <= 0 || h <= 0 || depth != 8 || interlace != 0) return false;
    if (w > 32768 || h > 32768) return false;  // corrupt or hostile header: no multi-GB allocation
    const int fch = ct == 0 ? 1 : (ct == 2 ? 3 : (ct == 3 ? 1 : (ct == 4 ? 2 : (ct == 6 ? 4 : 0))));
    if (!fch) return false;
    const size_t stride = (size_t)w * fch;
    std::vector<uint8_t> raw((stride + 1) * h);
    uLongf rl = (uLongf)raw.size();
    if (uncompress(raw.data(), &rl, idat.data(), (uLong)idat.size()) != Z_OK || rl != raw.size()) return false;
    std::vector<uint8_t> img(stride * h);
    for (int y = 0; y < h; ++y) {
        const uint8_t ft = raw[y * (stride + 1)];
        const uint8_t *src = &raw[y * (stride + 1) + 1];
        uint8_t *dst = &img[y * stride];
        const uint8_t *up = y > 0 ? &img[(y - 1) * stride] : nullptr;
        for (size_t i = 0; i < stride; ++i) {
            const int a = i >= (size_t)fch ? dst[i - fch] : 0, b = up ? up[i] : 0;
            const int c = (up && i >= (size_t)fch) ? up[i - fch] : 0;
            int v = src[i];
            switch (ft) {
                case 0: break;
                case 1: v += a; break;
                case 2: v += b; break;
                case 3: v += (a + b) / 2; break;
                case 4: v += paeth(a, b, c); break;
                default: return false;
            }
            dst[i] = (uint8_t)v;
        }
    }
    im.w = w;
    im.h = h;
    if (ct == 3) {  // palette -> RGB
        im.ch = 3;
        im.px.resize((size_t)w * h * 3);
        for (size_t i = 0; i < (size_t)w * h; ++i) {
            const size_t k = (size_t)img[i] * 3;
            for (int c = 0; c < 3; ++c) im.px[i * 3 + c] = k + c < plte.size() ? plte[k + c] : 0;
        }
    } else {
        im.ch = fch;
        im.px.swap(img);
    }
    return true;
}

// ImageDiff (ImageDiff.cpp): same arithmetic, same summation order
int count_different(const Image &a, const Image &b, float threshold) {
    int diff = 0;
    const int ch = std::min(a.ch, b.ch);
    for (int y = 0; y < a.h; y++)
        for (int x = 0; x < a.w; x++) {
            const int idx = y * a.w + x;
            for (int c = 0; c < ch; c++) {
                const float d = std::abs(static_cast<float>(a.px[idx * a.ch + c]) -
                                         static_cast<float>(b.px[idx * b.ch + c])) / 255.0f;
                if (d > threshold) { diff++; break; }
            }
        }
    return diff;
}
float rmse(const Image &a, const Image &b) {
    double sum = 0.0;
    int samples = 0;
    const int ch = std::min(a.ch, b.ch);
    for (int y = 0; y < a.h; y++)
        for (int x = 0; x < a.w; x++) {
            const int idx = y * a.w + x;
            for (int c = 0; c < ch; c++) {
                const double d = static_cast<double>(a.px[idx * a.ch + c]) - static_cast<double>(b.px[idx * b.ch + c]);
                sum += d * d;
                samples++;
            }
        }
    return static_cast<float>(std::sqrt(sum / samples));
}
std::vector<float> gray(const Image &im) {
    std::vector<float> g((size_t)im.w * im.h);
    for (int y = 0; y < im.h; y++)
        for (int x = 0; x < im.w; x++) {
            const int idx = y * im.w + x, p = idx * im.ch;
            g[idx] = im.ch >= 3 ? 0.299f * im.px[p] + 0.587f * im.px[p + 1] + 0.114f * im.px[p + 2] : im.px[p];
        }
    return g;
}
std::vector<float> gauss3(const std::vector<float> &im, int w, int h) {
    const float k[3][3] = {{1.0f / 16, 2.0f / 16, 1.0f / 16}, {2.0f / 16, 4.0f / 16, 2.0f / 16},
                           {1.0f / 16, 2.0f / 16, 1.0f / 16}};
    std::vector<float> out((size_t)w * h);
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            float s = 0.0f;
            for (int ky = -1; ky <= 1; ky++)
                for (int kx = -1; kx <= 1; kx++) {
                    const int ny = std::max(0, std::min(h - 1, y + ky)), nx = std::max(0, std::min(w - 1, x + kx));
                    s += im[ny * w + nx] * k[ky + 1][kx + 1];
                }
            out[y * w + x] = s;
        }
    return out;
}
float ssim(const Image &a, const Image &b) {
    const std::vector<float> ga = gauss3(gray(a), a.w, a.h), gb = gauss3(gray(b), b.w, b.h);
    const float K1 = 0.01f, K2 = 0.03f, L = 255.0f, C1 = (K1 * L) * (K1 * L), C2 = (K2 * L) * (K2 * L);
    auto mean = [](const std::vector<float> &v) {
        float s = 0.0f;
        for (float x : v) s += x;
        return s / v.size();
    };
    const float ma = mean(ga), mb = mean(gb);
    float va = 0.0f, vb = 0.0f, cov = 0.0f;
    for (float x : ga) { const float d = x - ma; va += d * d; }
    for (float x : gb) { const float d = x - mb; vb += d * d; }
    for (size_t i = 0; i < ga.size(); i++) cov += (ga[i] - ma) * (gb[i] - mb);
    va /= (ga.size() - 1);
    vb /= (gb.size() - 1);
    cov /= (ga.size() - 1);
    const float num = (2 * ma * mb + C1) * (2 * cov + C2);
    const float den = (ma * ma + mb * mb + C1) * (va + vb + C2);
    return num / den;
}

}  // namespace

namespace vx {
// PNG decode for the texture loader (8-bit grey / grey+alpha / RGB / RGBA / palette -> RGB)
bool decode_png(const std::string &path, int &w, int &h, int &ch, std::vector<uint8_t> &px) {
    Image im;
    if (!read_png(path, im)) return false;
    w = im.w;
    h = im.h;
    ch = im.ch;
    px.swap(im.px);
    return true;
}
}  // namespace vx

extern "C" {

int vxpt_write_png_rgba32f(const char *path, int w, int h, const float *rgba) {
    if (!path || !rgba || w <= 0 || h <= 0) return VXPT_ERR_ARG;
    Image im;
    im.w = w; im.h = h; im.ch = 3;
    im.px.resize((size_t)w * h * 3);
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            const float *p = rgba + ((size_t)y * w + x) * 4;
            uint8_t *d = &im.px[((size_t)(h - 1 - y) * w + x) * 3];  // flip Y
            for (int c = 0; c < 3; c++) d[c] = (unsigned char)(std::min(1.0f, std::max(0.0f, p[c])) * 255.0f);
        }
    return write_png(path, im) ? VXPT_OK : VXPT_ERR_IO;
}

int vxpt_read_png(const char *path, int *w, int *h, int *channels, uint8_t *pixels, size_t cap) {
    if (!path) return VXPT_ERR_ARG;
    Image im;
    if (!read_png(path, im)) return VXPT_ERR_IO;
    if (w) *w = im.w;
    if (h) *h = im.h;
    if (channels) *channels = im.ch;
    if (pixels) {
        if (cap < im.px.size()) return VXPT_ERR_ARG;
        std::memcpy(pixels, im.px.data(), im.px.size());
    }
    return VXPT_OK;
}

int vxpt_image_diff(const char *a, const char *b, vxpt_image_diff_result *out) {
    if (!a || !b || !out) return VXPT_ERR_ARG;
    Image ia, ib;
    if (!read_png(a, ia) || !read_png(b, ib)) return VXPT_ERR_IO;
    std::memset(out, 0, sizeof(*out));
    if (ia.w != ib.w || ia.h != ib.h) return VXPT_ERR_ARG;
    out->total_pixels = ia.w * ia.h;
    out->different_pixels = count_different(ia, ib, 0.01f);
    out->pixel_difference_ratio = static_cast<float>(out->different_pixels) / out->total_pixels;
    out->rmse = rmse(ia, ib);
    out->ssim = ssim(ia, ib);
    out->is_identical = out->different_pixels == 0;
    out->is_very_close = out->ssim > 0.99f && out->rmse < 1.0f;
    out->is_close = out->ssim > 0.95f && out->rmse < 5.0f;
    return VXPT_OK;
}

int vxpt_image_diff_png(const char *a, const char *b, const char *diff_png) {
    if (!a || !b || !diff_png) return VXPT_ERR_ARG;
    Image ia, ib;
    if (!read_png(a, ia) || !read_png(b, ib)) return VXPT_ERR_IO;
    if (ia.w != ib.w || ia.h != ib.h) return VXPT_ERR_ARG;
    Image d;
    d.w = ia.w; d.h = ia.h; d.ch = 3;
    d.px.resize((size_t)d.w * d.h * 3);
    const int ch = std::min(ia.ch, ib.ch);
    for (int i = 0; i < d.w * d.h; i++) {
        float dr = 0, dg = 0, db = 0;
        const int pa = i * ia.ch, pb = i * ib.ch;
        if (ch >= 1) dr = std::abs(static_cast<int>(ia.px[pa]) - static_cast<int>(ib.px[pb]));
        if (ch >= 2) dg = std::abs(static_cast<int>(ia.px[pa + 1]) - static_cast<int>(ib.px[pb + 1]));
        if (ch >= 3) db = std::abs(static_cast<int>(ia.px[pa + 2]) - static_cast<int>(ib.px[pb + 2]));
        else { dg = dr; db = dr; }
        d.px[i * 3] = static_cast<uint8_t>(std::min(255.0f, dr * 3.0f));
        d.px[i * 3 + 1] = static_cast<uint8_t>(std::min(255.0f, dg * 3.0f));
        d.px[i * 3 + 2] = static_cast<uint8_t>(std::min(255.0f, db * 3.0f));
    }
    return write_png(diff_png, d) ? VXPT_OK : VXPT_ERR_IO;
}

}  // extern "C"
