// png.cpp — minimal RGBA8 PNG encoder (the reference saves with image 0.25's RgbaImage::save,
// main.rs:774). Deflate "stored" blocks: exact pixels, no compression dependency.
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/yart_host.h"

namespace {
uint32_t crc_table[256];
bool crc_init = false;
void init_crc() {
  for (uint32_t n = 0; n < 256; ++n) {
    uint32_t c = n;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    crc_table[n] = c;
  }
  crc_init = true;
}
uint32_t crc32(const uint8_t* p, size_t n, uint32_t c = 0xFFFFFFFFu) {
  for (size_t i = 0; i < n; ++i) c = crc_table[(c ^ p[i]) & 0xFF] ^ (c >> 8);
  return c;
}
void put32(std::vector<uint8_t>& v, uint32_t x) {
  v.push_back((uint8_t)(x >> 24)); v.push_back((uint8_t)(x >> 16)); v.push_back((uint8_t)(x >> 8)); v.push_back((uint8_t)x);
}
void chunk(std::vector<uint8_t>& out, const char* type, const std::vector<uint8_t>& data) {
  put32(out, (uint32_t)data.size());
  size_t start = out.size();
  out.insert(out.end(), type, type + 4);
  out.insert(out.end(), data.begin(), data.end());
  put32(out, crc32(out.data() + start, out.size() - start) ^ 0xFFFFFFFFu);
}
}  // namespace

extern "C" int yart_write_png(const char* path, const uint8_t* rgba, uint32_t w, uint32_t h) {
  if (!path || !rgba || !w || !h) return YART_ERR_INVALID;
  if (!crc_init) init_crc();
  std::vector<uint8_t> raw;
  raw.reserve((size_t)h * (4 * (size_t)w + 1));
  for (uint32_t y = 0; y < h; ++y) {
    raw.push_back(0);  // filter: none
    raw.insert(raw.end(), rgba + (size_t)y * w * 4, rgba + (size_t)(y + 1) * w * 4);
  }
  std::vector<uint8_t> z = {0x78, 0x01};
  uint32_t a = 1, b = 0;
  for (uint8_t c : raw) { a = (a + c) % 65521u; b = (b + a) % 65521u; }
  for (size_t off = 0; off < raw.size() || off == 0;) {
    size_t n = raw.size() - off;
    if (n > 65535) n = 65535;
    bool last = off + n == raw.size();
    z.push_back(last ? 1 : 0);
    z.push_back((uint8_t)n); z.push_back((uint8_t)(n >> 8));
    z.push_back((uint8_t)~n); z.push_back((uint8_t)(~n >> 8));
    z.insert(z.end(), raw.begin() + off, raw.begin() + off + n);
    off += n;
    if (last) break;
  }
  put32(z, (b << 16) | a);
  std::vector<uint8_t> out = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
  std::vector<uint8_t> ihdr;
  put32(ihdr, w); put32(ihdr, h);
  ihdr.push_back(8); ihdr.push_back(6); ihdr.push_back(0); ihdr.push_back(0); ihdr.push_back(0);
  chunk(out, "IHDR", ihdr);
  chunk(out, "IDAT", z);
  chunk(out, "IEND", {});
  FILE* f = std::fopen(path, "wb");
  if (!f) return YART_ERR_IO;
  size_t wr = std::fwrite(out.data(), 1, out.size(), f);
  std::fclose(f);
  return wr == out.size() ? YART_OK : YART_ERR_IO;
}
