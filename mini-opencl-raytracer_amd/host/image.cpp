// image.cpp -- output/format step (include/rt_image.h): accumulation buffer -> PPM / PNG.
#include <cstdint>
#include <climits>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/rt_image.h"
#include "../../include/rt_status.h"

namespace {

inline unsigned char to8(float v) {
    if (!(v > 0.0f)) return 0;  // negative, zero and NaN
    if (v >= 1.0f) return 255;
    return (unsigned char)(v * 255.0f + 0.5f);
}

uint32_t crc32(const unsigned char* p, size_t n, uint32_t c = 0xffffffffu) {
    static uint32_t table[256];
    static bool init = false;
    if (!init) {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t k = i;
            for (int j = 0; j < 8; ++j) k = (k & 1u) ? 0xedb88320u ^ (k >> 1) : k >> 1;
            table[i] = k;
        }
        init = true;
    }
    for (size_t i = 0; i < n; ++i) c = table[(c ^ p[i]) & 0xffu] ^ (c >> 8);
    return c;
}

void put32(std::vector<unsigned char>& v, uint32_t x) {
    v.push_back((unsigned char)(x >> 24));
    v.push_back((unsigned char)(x >> 16));
    v.push_back((unsigned char)(x >> 8));
    v.push_back((unsigned char)x);
}

void chunk(std::FILE* f, const char* type, const std::vector<unsigned char>& data) {
    std::vector<unsigned char> c;
    put32(c, (uint32_t)data.size());
    c.insert(c.end(), type, type + 4);
    c.insert(c.end(), data.begin(), data.end());
    const uint32_t crc = crc32(c.data() + 4, c.size() - 4) ^ 0xffffffffu;
    put32(c, crc);
    std::fwrite(c.data(), 1, c.size(), f);
}

int check_args(const void* path, const float* px, unsigned W, unsigned H) {
    if (!path || !px || W == 0 || H == 0) return RT_INVALID_VALUE;
    if ((uint64_t)W * H * 3 > (1ull << 40)) return RT_INVALID_VALUE;
    return RT_SUCCESS;
}

}  // namespace

extern "C" int rtiToRGB8(const float* px, unsigned W, unsigned H, unsigned char* out) {
    if (!px || !out || W == 0 || H == 0) return RT_INVALID_VALUE;
    for (unsigned y = 0; y < H; ++y) {
        const float* src = px + 4 * (size_t)(H - 1 - y) * W;
        unsigned char* dst = out + 3 * (size_t)y * W;
        for (unsigned x = 0; x < W; ++x)
            for (int c = 0; c < 3; ++c) dst[3 * x + c] = to8(src[4 * x + c]);
    }
    return RT_SUCCESS;
}

extern "C" int rtiWritePPM(const char* path, const float* px, unsigned W, unsigned H) {
    int rc = check_args(path, px, W, H);
    if (rc) return rc;
    std::vector<unsigned char> rgb((size_t)W * H * 3);
    rtiToRGB8(px, W, H, rgb.data());
    std::FILE* f = std::fopen(path, "wb");
    if (!f) return RT_INVALID_VALUE;
    std::fprintf(f, "P6\n%u %u\n255\n", W, H);
    const bool ok = std::fwrite(rgb.data(), 1, rgb.size(), f) == rgb.size();
    return (std::fclose(f) == 0 && ok) ? RT_SUCCESS : RT_OUT_OF_RESOURCES;
}

extern "C" int rtiWritePNG(const char* path, const float* px, unsigned W, unsigned H) {
    int rc = check_args(path, px, W, H);
    if (rc) return rc;
    std::vector<unsigned char> rgb((size_t)W * H * 3);
    rtiToRGB8(px, W, H, rgb.data());
    // raw scanlines: filter byte 0 + RGB
    std::vector<unsigned char> raw;
    raw.reserve((size_t)H * (1 + 3 * (size_t)W));
    for (unsigned y = 0; y < H; ++y) {
        raw.push_back(0);
        raw.insert(raw.end(), rgb.begin() + 3 * (size_t)y * W, rgb.begin() + 3 * (size_t)(y + 1) * W);
    }
    // zlib: header, stored deflate blocks (<= 65535 bytes), Adler-32
    std::vector<unsigned char> z = {0x78, 0x01};
    size_t pos = 0;
    do {
        const size_t n = std::min<size_t>(65535, raw.size() - pos);
        const bool last = pos + n == raw.size();
        z.push_back(last ? 1 : 0);
        z.push_back((unsigned char)(n & 0xff));
        z.push_back((unsigned char)(n >> 8));
        z.push_back((unsigned char)(~n & 0xff));
        z.push_back((unsigned char)((~n >> 8) & 0xff));
        z.insert(z.end(), raw.begin() + pos, raw.begin() + pos + n);
        pos += n;
    } while (pos < raw.size());
    uint32_t a = 1, b = 0;
    for (unsigned char c : raw) {
        a = (a + c) % 65521u;
        b = (b + a) % 65521u;
    }
    put32(z, (b << 16) | a);

    std::FILE* f = std::fopen(path, "wb");
    if (!f) return RT_INVALID_VALUE;
    static const unsigned char sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    std::fwrite(sig, 1, 8, f);
    std::vector<unsigned char> ihdr;
    put32(ihdr, W);
    put32(ihdr, H);
    ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});  // 8-bit, RGB, deflate, filter 0, no interlace
    chunk(f, "IHDR", ihdr);
    chunk(f, "IDAT", z);
    chunk(f, "IEND", {});
    return std::fclose(f) == 0 ? RT_SUCCESS : RT_OUT_OF_RESOURCES;
}

// ---- accumulation checkpoint (rtiSaveAccum / rtiLoadAccum) ----------------------------------
namespace {

constexpr char kAccumMagic[8] = {'R', 'T', 'A', 'C', 'C', 'U', 'M', '1'};

uint64_t fnv1a64(const void* p, size_t n, uint64_t h) {
    const unsigned char* b = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; ++i) {
        h ^= b[i];
        h *= 1099511628211ull;
    }
    return h;
}

}  // namespace

extern "C" int rtiSaveAccum(const char* path, const float* px, unsigned W, unsigned H, unsigned next_frame) {
    if (!path || !px || W == 0 || H == 0) return RT_INVALID_VALUE;
    const uint32_t hdr[3] = {W, H, next_frame};
    const size_t bytes = (size_t)W * H * 16;
    uint64_t h = 14695981039346656037ull;
    h = fnv1a64(kAccumMagic, 8, h);
    h = fnv1a64(hdr, sizeof(hdr), h);
    h = fnv1a64(px, bytes, h);
    std::FILE* f = std::fopen(path, "wb");
    if (!f) return RT_INVALID_VALUE;
    bool ok = std::fwrite(kAccumMagic, 1, 8, f) == 8 && std::fwrite(hdr, sizeof(hdr), 1, f) == 1 &&
              std::fwrite(px, 1, bytes, f) == bytes && std::fwrite(&h, sizeof(h), 1, f) == 1;
    ok = (std::fclose(f) == 0) && ok;
    return ok ? RT_SUCCESS : RT_OUT_OF_RESOURCES;
}

extern "C" int rtiLoadAccum(const char* path, float* px, unsigned* W, unsigned* H, unsigned* next_frame) {
    if (!path || !W || !H || !next_frame) return RT_INVALID_VALUE;
    std::FILE* f = std::fopen(path, "rb");
    if (!f) return RT_FILE_NOT_FOUND;
    char magic[8];
    uint32_t hdr[3];
    int rc = RT_SUCCESS;
    if (std::fread(magic, 1, 8, f) != 8 || std::memcmp(magic, kAccumMagic, 8) != 0 ||
        std::fread(hdr, sizeof(hdr), 1, f) != 1 || hdr[0] == 0 || hdr[1] == 0)
        rc = RT_PARSE_ERROR;
    // W * H * 16 bytes must not wrap (a crafted W = H = 2^30 would make it 0 and let a 28-byte file
    // through, then a caller sizing W * H * 16 itself overflows too), and must fit a file offset
    size_t bytes = 0;
    if (!rc && (__builtin_mul_overflow((size_t)hdr[0], (size_t)hdr[1], &bytes) ||
                __builtin_mul_overflow(bytes, (size_t)16, &bytes) || bytes > (size_t)LONG_MAX - 64))
        rc = RT_PARSE_ERROR;
    if (!rc) {
        // the file holds exactly header + pixels + checksum
        if (std::fseek(f, 0, SEEK_END) != 0 || std::ftell(f) != (long)(8 + sizeof(hdr) + bytes + 8) ||
            std::fseek(f, 8 + sizeof(hdr), SEEK_SET) != 0)
            rc = RT_PARSE_ERROR;
    }
    if (!rc && px) {
        if (hdr[0] != *W || hdr[1] != *H) {
            rc = RT_INVALID_VALUE;
        } else {
            uint64_t stored = 0, h = 14695981039346656037ull;
            if (std::fread(px, 1, bytes, f) != bytes || std::fread(&stored, sizeof(stored), 1, f) != 1) {
                rc = RT_PARSE_ERROR;
            } else {
                h = fnv1a64(kAccumMagic, 8, h);
                h = fnv1a64(hdr, sizeof(hdr), h);
                h = fnv1a64(px, bytes, h);
                if (h != stored) rc = RT_PARSE_ERROR;
            }
        }
    }
    std::fclose(f);
    if (rc) return rc;
    *W = hdr[0];
    *H = hdr[1];
    *next_frame = hdr[2];
    return RT_SUCCESS;
}

