// file_io.cpp — photon text files and PNG output for the drop-in boundary (B1).
//
//  * pm_photons_write_txt: photon-mapping/src/hostCode.cu:31-49
//    (writeAlivePhotons: std::fixed, setprecision(6), "pos dir color" per line)
//  * pm_photons_read_txt: ray-tracer/src/hostCode.cu:26-52 (readPhotonsFromFile:
//    9 floats per record via operator>>; a missing file -> 0 photons + stderr)
//  * pm_write_png_rgba: stbi_write_png(path, W, H, 4, fb, W*4)
//    (ray-tracer/src/hostCode.cu:239-240), zlib-compressed RGBA8.
#include <zlib.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../../include/pm.h"

extern "C" void pm_free(void* p) { std::free(p); }

extern "C" int pm_photons_write_txt(const char* path, const pm_photon* ph, int64_t n) {
  if (!path || (n > 0 && !ph) || n < 0) return PM_ERR_INVALID;
  FILE* f = std::fopen(path, "w");
  if (!f) {
    std::fprintf(stderr, "Error opening file: %s\n", path);
    return PM_ERR_IO;
  }
  std::vector<char> buf(1 << 20);
  std::setvbuf(f, buf.data(), _IOFBF, buf.size());
  for (int64_t i = 0; i < n; i++) {
    const pm_photon& p = ph[i];
    // operator<< on float with std::fixed + precision 6 == printf("%.6f") of the
    // value promoted to double
    std::fprintf(f, "%.6f %.6f %.6f %.6f %.6f %.6f %.6f %.6f %.6f\n", (double)p.pos.x, (double)p.pos.y,
                 (double)p.pos.z, (double)p.dir.x, (double)p.dir.y, (double)p.dir.z, (double)p.color.x,
                 (double)p.color.y, (double)p.color.z);
  }
  std::fclose(f);
  return PM_OK;
}

extern "C" int pm_photons_read_txt(const char* path, pm_photon** out, int64_t* n) {
  if (!path || !out || !n) return PM_ERR_INVALID;
  *out = nullptr;
  *n = 0;
  FILE* f = std::fopen(path, "r");
  if (!f) {
    std::fprintf(stderr, "Error opening file: %s\n", path);
    return PM_OK;   // reference: count = 0, nullptr, continue
  }
  size_t cap = 1024, cnt = 0;
  pm_photon* v = (pm_photon*)std::malloc(cap * sizeof(pm_photon));
  float x[9];
  for (;;) {
    // operator>> for float: strtof semantics on whitespace-separated tokens
    int got = std::fscanf(f, "%f %f %f %f %f %f %f %f %f", &x[0], &x[1], &x[2], &x[3], &x[4], &x[5], &x[6],
                          &x[7], &x[8]);
    if (got != 9) break;
    if (cnt == cap) {
      cap *= 2;
      v = (pm_photon*)std::realloc(v, cap * sizeof(pm_photon));
    }
    pm_photon& p = v[cnt++];
    p.pos = {x[0], x[1], x[2]};
    p.dir = {x[3], x[4], x[5]};
    p.power = 0;
    p.color = {x[6], x[7], x[8]};
  }
  std::fclose(f);
  if (cnt == 0) {
    std::free(v);
    return PM_OK;
  }
  *out = v;
  *n = (int64_t)cnt;
  return PM_OK;
}

extern "C" int pm_photons_write_bin(const char* path, const pm_photon* ph, int64_t n) {
  if (!path || (n > 0 && !ph) || n < 0) return PM_ERR_INVALID;
  FILE* f = std::fopen(path, "wb");
  if (!f) return PM_ERR_IO;
  const char magic[8] = {'P', 'M', 'P', 'H', 'O', 'T', 'N', '1'};
  bool ok = std::fwrite(magic, 1, 8, f) == 8 && std::fwrite(&n, sizeof(n), 1, f) == 1 &&
            (n == 0 || std::fwrite(ph, sizeof(pm_photon), (size_t)n, f) == (size_t)n);
  ok = (std::fclose(f) == 0) && ok;
  return ok ? PM_OK : PM_ERR_IO;
}

extern "C" int pm_photons_read_bin(const char* path, pm_photon** out, int64_t* n) {
  if (!path || !out || !n) return PM_ERR_INVALID;
  *out = nullptr;
  *n = 0;
  FILE* f = std::fopen(path, "rb");
  if (!f) return PM_ERR_IO;
  char magic[8];
  int64_t cnt = 0;
  if (std::fread(magic, 1, 8, f) != 8 || std::memcmp(magic, "PMPHOTN1", 8) != 0 ||
      std::fread(&cnt, sizeof(cnt), 1, f) != 1 || cnt < 0) {
    std::fclose(f);
    return PM_ERR_IO;
  }
  pm_photon* v = cnt ? (pm_photon*)std::malloc((size_t)cnt * sizeof(pm_photon)) : nullptr;
  if (cnt && (!v || std::fread(v, sizeof(pm_photon), (size_t)cnt, f) != (size_t)cnt)) {
    std::free(v);
    std::fclose(f);
    return PM_ERR_IO;
  }
  std::fclose(f);
  *out = v;
  *n = cnt;
  return PM_OK;
}

namespace {
void put32(std::vector<unsigned char>& o, uint32_t v) {
  o.push_back((unsigned char)(v >> 24));
  o.push_back((unsigned char)(v >> 16));
  o.push_back((unsigned char)(v >> 8));
  o.push_back((unsigned char)v);
}
void chunk(std::vector<unsigned char>& o, const char* type, const unsigned char* data, size_t len) {
  put32(o, (uint32_t)len);
  const size_t start = o.size();
  o.insert(o.end(), type, type + 4);
  if (len) o.insert(o.end(), data, data + len);
  uint32_t crc = (uint32_t)crc32(0L, o.data() + start, (uInt)(len + 4));
  put32(o, crc);
}
}  // namespace

extern "C" int pm_write_png_rgba(const char* path, const uint32_t* rgba, int32_t w, int32_t h) {
  if (!path || !rgba || w <= 0 || h <= 0) return PM_ERR_INVALID;
  // raw scanlines, filter type 0; uint32 0xAABBGGRR little-endian == bytes R,G,B,A
  std::vector<unsigned char> raw((size_t)h * ((size_t)w * 4 + 1));
  for (int32_t y = 0; y < h; y++) {
    unsigned char* row = &raw[(size_t)y * ((size_t)w * 4 + 1)];
    row[0] = 0;
    std::memcpy(row + 1, rgba + (size_t)y * w, (size_t)w * 4);
  }
  uLongf zlen = compressBound((uLong)raw.size());
  std::vector<unsigned char> z(zlen);
  if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 6) != Z_OK) return PM_ERR_IO;
  std::vector<unsigned char> o = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
  unsigned char ihdr[13];
  const uint32_t W = (uint32_t)w, H = (uint32_t)h;
  ihdr[0] = (unsigned char)(W >> 24); ihdr[1] = (unsigned char)(W >> 16); ihdr[2] = (unsigned char)(W >> 8); ihdr[3] = (unsigned char)W;
  ihdr[4] = (unsigned char)(H >> 24); ihdr[5] = (unsigned char)(H >> 16); ihdr[6] = (unsigned char)(H >> 8); ihdr[7] = (unsigned char)H;
  ihdr[8] = 8;   // bit depth
  ihdr[9] = 6;   // RGBA
  ihdr[10] = ihdr[11] = ihdr[12] = 0;
  chunk(o, "IHDR", ihdr, 13);
  chunk(o, "IDAT", z.data(), zlen);
  chunk(o, "IEND", nullptr, 0);
  FILE* f = std::fopen(path, "wb");
  if (!f) return PM_ERR_IO;
  const size_t wr = std::fwrite(o.data(), 1, o.size(), f);
  std::fclose(f);
  return wr == o.size() ? PM_OK : PM_ERR_IO;
}
