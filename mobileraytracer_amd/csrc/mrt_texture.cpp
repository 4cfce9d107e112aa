// mrt_texture.cpp - PNG decoding for material textures (map_Kd).
//
// The reference decodes textures with stb_image (Texture.cpp:83-114, stbi_load_from_memory with
// req_comp = 0), which is not in the image; this is a restatement of the part of that decoder
// the reference's scenes reach: non-interlaced PNG of every colour type and bit depth, with
// stb_image's output conventions - 8 bits per channel, palette images expanded to RGB (RGBA
// with a tRNS chunk), a tRNS key adding an alpha channel to grey / RGB images, grey depths
// below 8 scaled to 0..255 (x 0xFF / 0x55 / 0x11), 16-bit samples reduced to their high byte.
#include "mrt_scene.hpp"

#include <zlib.h>

#include <cstring>
#include <fstream>
#include <iterator>

namespace mrt {

namespace {

uint32_t be32(const uint8_t* p) {
    return (static_cast<uint32_t>(p[0]) << 24) | (static_cast<uint32_t>(p[1]) << 16) | (static_cast<uint32_t>(p[2]) << 8) |
           static_cast<uint32_t>(p[3]);
}

int paeth(int a, int b, int c) {
    const int p = a + b - c;
    const int pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    if (pa <= pb && pa <= pc) return a;
    if (pb <= pc) return b;
    return c;
}

}  // namespace

bool decodePng(const std::vector<uint8_t>& file, HTexture* out, std::string* err) {
    static const uint8_t kSig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (file.size() < 8 || std::memcmp(file.data(), kSig, 8) != 0) {
        *err = "not a PNG file";
        return false;
    }
    uint32_t w = 0, h = 0;
    int depth = 0, ctype = -1, interlace = 0;
    std::vector<uint8_t> idat, palette, trns;
    size_t p = 8;
    bool ended = false;
    while (p + 12 <= file.size() && !ended) {
        const uint32_t len = be32(&file[p]);
        if (p + 12 + static_cast<size_t>(len) > file.size()) break;
        const uint8_t* type = &file[p + 4];
        const uint8_t* data = &file[p + 8];
        if (std::memcmp(type, "IHDR", 4) == 0 && len >= 13) {
            w = be32(data);
            h = be32(data + 4);
            depth = data[8];
            ctype = data[9];
            interlace = data[12];
        } else if (std::memcmp(type, "PLTE", 4) == 0) {
            palette.assign(data, data + len);
        } else if (std::memcmp(type, "tRNS", 4) == 0) {
            trns.assign(data, data + len);
        } else if (std::memcmp(type, "IDAT", 4) == 0) {
            idat.insert(idat.end(), data, data + len);
        } else if (std::memcmp(type, "IEND", 4) == 0) {
            ended = true;
        }
        p += 12 + static_cast<size_t>(len);
    }
    const int chans = ctype == 0 ? 1 : ctype == 2 ? 3 : ctype == 3 ? 1 : ctype == 4 ? 2 : ctype == 6 ? 4 : 0;
    if (w == 0 || h == 0 || chans == 0 || w > (1u << 16) || h > (1u << 16)) {
        *err = "unsupported PNG header";
        return false;
    }
    if (interlace != 0) {
        *err = "interlaced PNG is not supported";
        return false;
    }
    if (!(depth == 1 || depth == 2 || depth == 4 || depth == 8 || depth == 16) || (ctype == 3 && depth == 16) ||
        ((ctype == 2 || ctype == 4 || ctype == 6) && depth < 8)) {
        *err = "unsupported PNG bit depth";
        return false;
    }
    const size_t rowBytes = (static_cast<size_t>(w) * static_cast<size_t>(chans) * static_cast<size_t>(depth) + 7) / 8;
    std::vector<uint8_t> raw((rowBytes + 1) * h);
    uLongf rawLen = static_cast<uLongf>(raw.size());
    if (uncompress(raw.data(), &rawLen, idat.data(), static_cast<uLong>(idat.size())) != Z_OK || rawLen != raw.size()) {
        *err = "corrupt PNG image data";
        return false;
    }
    // unfilter in place (filter bytes 0-4; the row above the first is zero)
    const int bpp = std::max(1, chans * depth / 8);
    std::vector<uint8_t> img(rowBytes * h);
    for (uint32_t y = 0; y < h; ++y) {
        const uint8_t f = raw[y * (rowBytes + 1)];
        const uint8_t* src = &raw[y * (rowBytes + 1) + 1];
        uint8_t* cur = &img[y * rowBytes];
        const uint8_t* prev = y > 0 ? &img[(y - 1) * rowBytes] : nullptr;
        for (size_t x = 0; x < rowBytes; ++x) {
            const int a = x >= static_cast<size_t>(bpp) ? cur[x - static_cast<size_t>(bpp)] : 0;
            const int b = prev != nullptr ? prev[x] : 0;
            const int c = (prev != nullptr && x >= static_cast<size_t>(bpp)) ? prev[x - static_cast<size_t>(bpp)] : 0;
            int v = src[x];
            switch (f) {
                case 0: break;
                case 1: v += a; break;
                case 2: v += b; break;
                case 3: v += (a + b) / 2; break;
                case 4: v += paeth(a, b, c); break;
                default: *err = "bad PNG filter"; return false;
            }
            cur[x] = static_cast<uint8_t>(v & 0xFF);
        }
    }
    // samples -> 8-bit channels with stb_image's conventions
    const bool hasTrns = !trns.empty();
    const int outC = ctype == 3 ? (hasTrns ? 4 : 3) : chans + ((hasTrns && (ctype == 0 || ctype == 2)) ? 1 : 0);
    out->width = static_cast<int32_t>(w);
    out->height = static_cast<int32_t>(h);
    out->channels = outC;
    out->texels.assign(static_cast<size_t>(w) * h * static_cast<size_t>(outC), 0);
    auto sample = [&](const uint8_t* row, size_t i) -> int {  // i-th sample of a row at this depth
        if (depth == 8) return row[i];
        if (depth == 16) return (row[2 * i] << 8) | row[2 * i + 1];
        const int perByte = 8 / depth;
        const int shift = 8 - depth * (1 + static_cast<int>(i % static_cast<size_t>(perByte)));
        return (row[i / static_cast<size_t>(perByte)] >> shift) & ((1 << depth) - 1);
    };
    const int scale = depth == 1 ? 0xFF : depth == 2 ? 0x55 : depth == 4 ? 0x11 : 1;
    for (uint32_t y = 0; y < h; ++y) {
        const uint8_t* row = &img[y * rowBytes];
        for (uint32_t x = 0; x < w; ++x) {
            uint8_t* o = &out->texels[(static_cast<size_t>(y) * w + x) * static_cast<size_t>(outC)];
            if (ctype == 3) {
                const int idx = sample(row, x);
                for (int k = 0; k < 3; ++k)
                    o[k] = (static_cast<size_t>(3 * idx + k) < palette.size()) ? palette[static_cast<size_t>(3 * idx + k)] : 0;
                if (outC == 4) o[3] = static_cast<size_t>(idx) < trns.size() ? trns[static_cast<size_t>(idx)] : 255;
                continue;
            }
            int s[4] = {0, 0, 0, 0};
            for (int k = 0; k < chans; ++k) s[k] = sample(row, static_cast<size_t>(x) * static_cast<size_t>(chans) + k);
            for (int k = 0; k < chans; ++k)
                o[k] = static_cast<uint8_t>(depth == 16 ? (s[k] >> 8) : (depth < 8 ? s[k] * scale : s[k]));
            if (outC == chans + 1) {  // tRNS key on grey / RGB
                bool key = true;
                for (int k = 0; k < chans; ++k) {
                    const size_t at = static_cast<size_t>(2 * k);
                    const int kv = at + 1 < trns.size() ? ((trns[at] << 8) | trns[at + 1]) : -1;
                    key = key && kv == s[k];
                }
                o[chans] = key ? 0 : 255;
            }
        }
    }
    return true;
}

bool loadTextureFile(const std::string& path, HTexture* out, std::string* err) {
    std::ifstream f(path, std::ios::binary);
    if (!f) {
        *err = "cannot open texture " + path;
        return false;
    }
    const std::vector<uint8_t> bytes((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    return decodePng(bytes, out, err);
}

}  // namespace mrt
