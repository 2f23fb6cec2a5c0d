/*
 * jxo_cli.c -- ORACLE command line (test infrastructure): encode a binary PPM
 * (P6, 8-bit) with the CPU restatement.  Mirrors the cjxl argv shape used by
 * benchmark-jpegxl/src/docker_manager.rs:126-136.
 *   jxo_cli in.ppm out.jxl --distance=D --effort=E [--proposals=none|P|F|PF]
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "jxo.h"

static uint8_t* read_ppm(const char* path, uint32_t* w, uint32_t* h) {
  FILE* f = fopen(path, "rb");
  if (!f) return NULL;
  char magic[3] = {0};
  unsigned mx;
  if (fscanf(f, "%2s %u %u %u", magic, w, h, &mx) != 4 || strcmp(magic, "P6") || mx != 255) {
    fclose(f);
    return NULL;
  }
  fgetc(f);
  size_t n = (size_t)(*w) * (*h) * 3;
  uint8_t* buf = (uint8_t*)malloc(n);
  if (fread(buf, 1, n, f) != n) {
    free(buf);
    buf = NULL;
  }
  fclose(f);
  return buf;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s in.ppm out.jxl --distance=D --effort=E\n", argv[0]);
    return 2;
  }
  jxo_params p = {1.0f, 7, 0, 0};
  for (int i = 3; i < argc; i++) {
    if (!strncmp(argv[i], "--distance=", 11)) p.distance = (float)atof(argv[i] + 11);
    else if (!strncmp(argv[i], "--effort=", 9)) p.effort = atoi(argv[i] + 9);
    else if (!strncmp(argv[i], "--proposals=", 12)) {
      const char* v = argv[i] + 12;
      p.proposals = (strchr(v, 'P') ? 1u : 0u) | (strchr(v, 'F') ? 2u : 0u);
    }
  }
  uint32_t w, h;
  uint8_t* rgb = read_ppm(argv[1], &w, &h);
  if (!rgb) {
    fprintf(stderr, "cannot read %s\n", argv[1]);
    return 1;
  }
  jxo_result r;
  int st = jxo_encode_rgb8(rgb, w, h, (size_t)w * 3, &p, &r);
  free(rgb);
  if (st) {
    fprintf(stderr, "encode failed: %d\n", st);
    return 1;
  }
  FILE* o = fopen(argv[2], "wb");
  if (!o || fwrite(r.bytes, 1, r.nbytes, o) != r.nbytes) {
    fprintf(stderr, "cannot write %s\n", argv[2]);
    return 1;
  }
  fclose(o);
  jxo_result_free(&r);
  return 0;
}
