/*
 * synth.c -- ORACLE (test infrastructure): the deterministic integer-only
 * synthetic RGB8 generator of SURVEY.md §8(d), a C restatement of
 * jxg/synth.py synth_rgb8 (same output bytes; tests/test_synth.py), with
 * OpenMP over rows.  The numpy version needs minutes at 16384^2.
 */
#include <stdint.h>

#include "jxo.h"

static inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  uint64_t z = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
/* numpy floor division of an int by a positive int */
static inline int floordiv(int a, int b) {
  const int q = a / b;
  return (a % b != 0 && a < 0) ? q - 1 : q;
}

void jxo_synth_rgb8(uint32_t w, uint32_t h, uint64_t seed, uint8_t* out) {
  const uint32_t ntx = (w + 63) / 64;
  const uint64_t nmul = seed * 0x100000001B3ull;
#pragma omp parallel for schedule(static)
  for (uint32_t y = 0; y < h; y++) {
    const int ly = (int)(y % 64);
    for (uint32_t x = 0; x < w; x++) {
      const int lx = (int)(x % 64);
      const uint64_t th = splitmix64(seed ^ (uint64_t)((y / 64) * ntx + x / 64));
      const int kind = (int)(th % 9);
      const int period = (int)(2 + (th >> 56) % 14);
      const int black = ((th >> 40) % 5) == 0;
      const uint64_t n64 = splitmix64(nmul ^ (((uint64_t)y << 32) | x));
      for (int c = 0; c < 3; c++) {
        const int c0 = (int)((th >> (8 + 8 * c)) & 0xFF), c1 = (int)((th >> (32 + 8 * c)) & 0xFF);
        const int noise = (int)((n64 >> (8 * c)) & 0xFF);
        const int hgrad = c0 + floordiv((c1 - c0) * lx, 63);
        const int vgrad = c0 + floordiv((c1 - c0) * ly, 63);
        int v;
        switch (kind) {
          case 0: v = black ? 0 : c0; break;
          case 1: v = hgrad; break;
          case 2: v = vgrad; break;
          case 3: v = ((ly / period) % 2 == 0) ? c0 : c1; break;
          case 4: v = ((lx / period) % 2 == 0) ? c0 : c1; break;
          case 5: v = (((lx / period + ly / period) % 2) == 0) ? c0 : c1; break;
          case 6: v = ((lx < 32) ^ (ly < 32)) ? c0 : c1; break;
          case 7: v = noise; break;
          default: v = floordiv(hgrad + vgrad, 2) + (noise % 17) - 8; break;
        }
        out[((size_t)y * w + x) * 3 + c] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
      }
    }
  }
}
