// jxg_cjxl -- cjxl-argv-compatible command line over the C ABI.
//
// The reference harness runs `cjxl IN OUT --distance=D --effort=E`
// (benchmark-jpegxl/src/docker_manager.rs:126-136) and maps a non-zero exit
// status to "skip" (benchmark.rs:654-677).  This tool accepts the same argv
// shape (plus --proposals=none|P|F|PF and --device=N), reads 8-bit PNG
// (gray / gray+alpha / RGB / RGBA, non-interlaced; alpha dropped) or binary
// PPM, encodes on the GPU and writes the codestream.  Exit 0 on success; a
// message on stderr and exit 1 otherwise.
#include <zlib.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/jxg.h"

namespace {

bool read_file(const char* path, std::vector<uint8_t>& out) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return false;
  std::fseek(f, 0, SEEK_END);
  long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  out.resize(n > 0 ? (size_t)n : 0);
  bool ok = n >= 0 && std::fread(out.data(), 1, out.size(), f) == out.size();
  std::fclose(f);
  return ok;
}

uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | p[1] << 16 | p[2] << 8 | p[3]; }

bool decode_png(const std::vector<uint8_t>& d, std::vector<uint8_t>& rgb, uint32_t& w,
                uint32_t& h, std::string& err) {
  static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  if (d.size() < 8 || std::memcmp(d.data(), sig, 8)) return err = "not a PNG", false;
  size_t p = 8;
  int depth = 0, ctype = -1, interlace = 0;
  std::vector<uint8_t> idat;
  while (p + 12 <= d.size()) {
    const uint32_t len = be32(&d[p]);
    const char* type = (const char*)&d[p + 4];
    if (p + 12 + (size_t)len > d.size()) return err = "truncated PNG", false;
    const uint8_t* body = &d[p + 8];
    if (!std::memcmp(type, "IHDR", 4)) {
      w = be32(body);
      h = be32(body + 4);
      depth = body[8];
      ctype = body[9];
      interlace = body[12];
    } else if (!std::memcmp(type, "IDAT", 4)) {
      idat.insert(idat.end(), body, body + len);
    } else if (!std::memcmp(type, "IEND", 4)) {
      break;
    }
    p += 12 + len;
  }
  if (depth != 8 || interlace || !(ctype == 0 || ctype == 2 || ctype == 4 || ctype == 6))
    return err = "unsupported PNG (need 8-bit, non-interlaced gray/RGB[A])", false;
  const int ch = ctype == 0 ? 1 : ctype == 2 ? 3 : ctype == 4 ? 2 : 4;
  const size_t stride = (size_t)w * ch;
  std::vector<uint8_t> raw((stride + 1) * h);
  uLongf rawlen = raw.size();
  if (uncompress(raw.data(), &rawlen, idat.data(), idat.size()) != Z_OK || rawlen != raw.size())
    return err = "PNG inflate failed", false;
  std::vector<uint8_t> img(stride * h), prev(stride, 0);
  for (uint32_t y = 0; y < h; y++) {
    const uint8_t ft = raw[y * (stride + 1)];
    const uint8_t* src = &raw[y * (stride + 1) + 1];
    uint8_t* row = &img[y * stride];
    for (size_t x = 0; x < stride; x++) {
      const int a = x >= (size_t)ch ? row[x - ch] : 0, b = prev[x],
                c = x >= (size_t)ch ? prev[x - ch] : 0;
      int v = src[x];
      switch (ft) {
        case 0: break;
        case 1: v += a; break;
        case 2: v += b; break;
        case 3: v += (a + b) / 2; break;
        case 4: {
          const int pp = a + b - c, pa = std::abs(pp - a), pb = std::abs(pp - b), pc = std::abs(pp - c);
          v += (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
          break;
        }
        default: return err = "bad PNG filter", false;
      }
      row[x] = (uint8_t)v;
    }
    std::memcpy(prev.data(), row, stride);
  }
  rgb.resize((size_t)w * h * 3);
  for (size_t i = 0; i < (size_t)w * h; i++)
    for (int c = 0; c < 3; c++) rgb[i * 3 + c] = img[i * ch + (ch >= 3 ? c : 0)];
  return true;
}

bool decode_ppm(const std::vector<uint8_t>& d, std::vector<uint8_t>& rgb, uint32_t& w,
                uint32_t& h, std::string& err) {
  std::string s(d.begin(), d.begin() + std::min<size_t>(d.size(), 64));
  unsigned W, H, M;
  int off = 0;
  if (std::sscanf(s.c_str(), "P6 %u %u %u%n", &W, &H, &M, &off) != 3 || M != 255)
    return err = "unsupported PPM", false;
  off += 1;
  w = W;
  h = H;
  if (d.size() < (size_t)off + (size_t)W * H * 3) return err = "truncated PPM", false;
  rgb.assign(d.begin() + off, d.begin() + off + (size_t)W * H * 3);
  return true;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr,
                 "usage: %s INPUT OUTPUT [--distance=D] [--effort=E] "
                 "[--proposals=none|P|F|PF] [--coder=ans|prefix] [--gaborish=1|0] "
                 "[--epf=-1|0] [--aq=masking|activity] [--device=N]\n"
                 "defaults: cjxl's (ANS, --gaborish=1, --epf=-1, masking AQ)\n",
                 argv[0]);
    return 1;
  }
  // `cjxl IN OUT --distance=D --effort=E` with no other flag (the harness's
  // argv, docker_manager.rs:126-136) gets cjxl's VarDCT defaults [ext]: ANS,
  // Gaborish on, EPF iterations by distance, the masking quant field
  jxg_params p{1.0f, 7, 0, 1, JXG_FLAGS_CJXL_DEFAULTS, 0};
  for (int i = 3; i < argc; i++) {
    const char* a = argv[i];
    if (!std::strncmp(a, "--distance=", 11) || !std::strncmp(a, "-d=", 3))
      p.distance = (float)std::atof(std::strchr(a, '=') + 1);
    else if (!std::strncmp(a, "--effort=", 9) || !std::strncmp(a, "-e=", 3))
      p.effort = std::atoi(std::strchr(a, '=') + 1);
    else if (!std::strncmp(a, "--proposals=", 12)) {
      const char* v = a + 12;
      p.proposals = (std::strchr(v, 'P') ? JXG_PROPOSAL_P : 0u) | (std::strchr(v, 'F') ? JXG_PROPOSAL_F : 0u);
    } else if (!std::strncmp(a, "--coder=", 8)) {
      if (!std::strcmp(a + 8, "prefix"))
        p.flags &= ~JXG_FLAG_ANS;
      else if (std::strcmp(a + 8, "ans")) {
        std::fprintf(stderr, "unknown coder: %s\n", a + 8);
        return 1;
      }
    } else if (!std::strncmp(a, "--gaborish=", 11)) {  // cjxl --gaborish
      if (!std::strcmp(a + 11, "0"))
        p.flags &= ~JXG_FLAG_GABORISH;
      else if (std::strcmp(a + 11, "1")) {
        std::fprintf(stderr, "unsupported --gaborish: %s\n", a + 11);
        return 1;
      }
    } else if (!std::strncmp(a, "--epf=", 6)) {  // cjxl --epf: -1 = by distance
      if (!std::strcmp(a + 6, "0"))
        p.flags &= ~JXG_FLAG_EPF;
      else if (std::strcmp(a + 6, "-1")) {
        std::fprintf(stderr, "unsupported --epf (-1 or 0): %s\n", a + 6);
        return 1;
      }
    } else if (!std::strncmp(a, "--aq=", 5)) {  // the quant field heuristic
      if (!std::strcmp(a + 5, "activity"))
        p.flags &= ~JXG_FLAG_AQ_MASKING;
      else if (std::strcmp(a + 5, "masking")) {
        std::fprintf(stderr, "unsupported --aq (masking or activity): %s\n", a + 5);
        return 1;
      }
    } else if (!std::strncmp(a, "--device=", 9))
      p.device = std::atoi(a + 9);
    else {
      std::fprintf(stderr, "unknown argument: %s\n", a);
      return 1;
    }
  }
  std::vector<uint8_t> file, rgb;
  if (!read_file(argv[1], file)) {
    std::fprintf(stderr, "cannot read %s\n", argv[1]);
    return 1;
  }
  uint32_t w = 0, h = 0;
  std::string err;
  const bool ok = file.size() >= 2 && file[0] == 'P' && file[1] == '6'
                      ? decode_ppm(file, rgb, w, h, err)
                      : decode_png(file, rgb, w, h, err);
  if (!ok) {
    std::fprintf(stderr, "%s: %s\n", argv[1], err.c_str());
    return 1;
  }
  jxg_ctx* ctx = nullptr;
  jxg_status st = jxg_create(&p, &ctx);
  if (st != JXG_OK) {
    std::fprintf(stderr, "jxg_create: %s\n", jxg_status_str(st));
    return 1;
  }
  jxg_buffer out{};
  const auto t0 = std::chrono::steady_clock::now();
  st = jxg_encode_rgb8(ctx, rgb.data(), w, h, (size_t)w * 3, &out);
  const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (st != JXG_OK) {
    std::fprintf(stderr, "encode failed: %s\n", jxg_status_str(st));
    jxg_destroy(ctx);
    return 1;
  }
  FILE* f = std::fopen(argv[2], "wb");
  if (!f || std::fwrite(out.data, 1, out.size, f) != out.size) {
    std::fprintf(stderr, "cannot write %s\n", argv[2]);
    if (f) std::fclose(f);
    jxg_buffer_free(&out);
    jxg_destroy(ctx);
    return 1;
  }
  std::fclose(f);
  std::printf("Encoding [VarDCT, d%.3f, effort: %d], %u x %u, %zu bytes, %.3f bpp, %.2f MP/s\n",
              p.distance, p.effort, w, h, out.size, out.size * 8.0 / ((double)w * h),
              (double)w * h / 1e6 / sec);
  jxg_buffer_free(&out);
  jxg_destroy(ctx);
  return 0;
}
