// CPU reference backend (see cpu_backend.hpp).
#include "heat/cpu_backend.hpp"

#include <omp.h>

#include <cmath>
#include <cstring>

#include "heat/common.hpp"
#include "heat/init_fn.hpp"

namespace heat::cpu {

void set_threads(int n) {
  if (n > 0) omp_set_num_threads(n);
}
int get_threads() { return omp_get_max_threads(); }

void init_field(float* origin, const Layout& L, int64_t gx0, int64_t gy0, int64_t nx, int64_t ny,
                int mode, uint64_t seed) {
  float* base = origin - L.origin();
#pragma omp parallel for schedule(static)
  for (int64_t r = 0; r < L.rows; ++r)
    for (int64_t c = 0; c < L.pitch; ++c)
      base[r * L.pitch + c] = init_value(mode, gx0 + r - L.hx, gy0 + c - L.hy, nx, ny, seed);
}

static inline bool interior(int64_t g, int64_t n) { return g >= 1 && g <= n - 2; }

float step(const float* src, float* dst, const Geom& g, const Box& box, bool want_resid) {
  if (box.empty()) return 0.0f;
  uint32_t mbits = 0;
  // Only the global-interior part of each row is updated; boundary cells are
  // copied so dst holds a complete field for the box.
  const int64_t cl = std::max(box.c0, 1 - g.gy0), ch = std::min(box.c1, g.ny - 1 - g.gy0);
#pragma omp parallel for schedule(static) reduction(max : mbits)
  for (int64_t r = box.r0; r < box.r1; ++r) {
    const float* s = src + r * g.pitch;
    float* d = dst + r * g.pitch;
    if (!interior(g.gx0 + r, g.nx) || cl >= ch) {
      std::memcpy(d + box.c0, s + box.c0, size_t(box.cols()) * 4);
      continue;
    }
    const float* n = s - g.pitch;
    const float* so = s + g.pitch;
    for (int64_t c = box.c0; c < cl; ++c) d[c] = s[c];
    uint32_t rm = 0;
    auto row = [&](auto update) {
      for (int64_t c = cl; c < ch; ++c) {
        const float v = update(s[c], n[c], so[c], s[c - 1], s[c + 1], g.cx, g.cy);
        d[c] = v;
        if (want_resid) {
          float diff = std::fabs(v - s[c]);
          uint32_t bits;
          std::memcpy(&bits, &diff, 4);
          rm = bits > rm ? bits : rm;
        }
      }
    };
    if (g.numerics == 1)
      row([](float c, float n, float s, float w, float e, float cx, float cy) {
        return stencil_mpi(c, n, s, w, e, cx, cy);
      });
    else
      row([](float c, float n, float s, float w, float e, float cx, float cy) {
        return stencil(c, n, s, w, e, cx, cy);
      });
    for (int64_t c = ch; c < box.c1; ++c) d[c] = s[c];
    mbits = rm > mbits ? rm : mbits;
  }
  float m;
  std::memcpy(&m, &mbits, 4);
  return want_resid ? m : 0.0f;
}

void copy_box(const float* src, int64_t src_pitch, float* dst, int64_t dst_pitch, const Box& box) {
  if (box.empty()) return;
#pragma omp parallel for schedule(static) if (box.rows() > 64)
  for (int64_t r = box.r0; r < box.r1; ++r)
    std::memcpy(dst + r * dst_pitch + box.c0, src + r * src_pitch + box.c0,
                size_t(box.cols()) * 4);
}

}  // namespace heat::cpu
