// Host-only self-test of the native engine's CPU components (topology,
// decomposition, layouts, prtdat formatting, initial condition, CPU stencil,
// deep-halo invariance).  Built twice: plain (`make selftest`) and under
// AddressSanitizer + UndefinedBehaviorSanitizer (`make selftest-asan`); the
// reference's latent OOB/UB bugs are the kind of thing
// the sanitizer build guards against here.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "heat/cpu_backend.hpp"
#include "heat/init_fn.hpp"
#include "heat/io.hpp"
#include "heat/topology.hpp"

using namespace heat;

static int failures = 0;
#define EXPECT(c)                                                      \
  do {                                                                 \
    if (!(c)) {                                                        \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                      \
    }                                                                  \
  } while (0)

static void test_dims() {
  const int want[][3] = {{1, 1, 1}, {2, 2, 1}, {6, 3, 2}, {8, 4, 2}, {10, 5, 2}, {12, 4, 3},
                         {16, 4, 4}, {7, 7, 1}, {36, 6, 6}};
  for (auto& w : want) {
    auto d = dims_create(w[0], 2);
    EXPECT(d[0] == w[1] && d[1] == w[2]);
  }
  auto d3 = dims_create(24, 3);
  EXPECT(d3[0] * d3[1] * d3[2] == 24 && d3[0] >= d3[1] && d3[1] >= d3[2]);
}

static void test_blocks() {
  for (int world : {1, 2, 3, 4, 6, 8}) {
    Cart c(world, DecompKind::Auto, 0, 0, 37, 53);
    int64_t cells = 0;
    for (int r = 0; r < world; ++r) {
      Block b = make_block(c, r, 37, 53);
      cells += b.lx * b.ly;
      auto n = c.neighbors(r);
      if (n[South] >= 0) EXPECT(make_block(c, n[South], 37, 53).ox == b.ox + b.lx);
      if (n[East] >= 0) EXPECT(make_block(c, n[East], 37, 53).oy == b.oy + b.ly);
    }
    EXPECT(cells == 37 * 53);
  }
  Layout L = Layout::make(7, 5, 3);
  EXPECT(L.pitch % 64 == 0 && L.hy == 4 && L.rows == 13 && L.origin() == 3 * L.pitch + 4);
}

static void test_format() {
  struct {
    float v;
    const char* s;
  } cases[] = {{0.f, "   0.0"}, {-0.f, "  -0.0"}, {0.25f, "   0.2"}, {0.75f, "   0.8"},
               {2.5f, "   2.5"}, {-12.34f, " -12.3"}, {123456.78f, "123456.8"},
               {-2147483648.f, "-2147483648.0"}};
  for (auto& c : cases) {
    std::string s;
    format_6_1f(c.v, s);
    EXPECT(s == c.s);
    char buf[64];
    std::snprintf(buf, sizeof buf, "%6.1f", double(c.v));
    EXPECT(s == buf);
  }
}

static void test_init_wrap() {
  // n = 1000 overflows int32: compare with explicit wrap-around arithmetic.
  const int64_t n = 1000;
  for (int64_t ix : {0L, 1L, 499L, 500L, 998L})
    for (int64_t iy : {0L, 3L, 500L, 997L}) {
      int64_t a = int32_t(uint32_t(ix * (n - ix - 1)));
      a = int32_t(uint32_t(a * iy));
      a = int32_t(uint32_t(a * (n - iy - 1)));
      EXPECT(init_ref_wrap(ix, iy, n, n) == float(int32_t(a)));
    }
  EXPECT(init_value(0, -1, 5, n, n, 0) == 0.f);
}

static void test_cpu_step_and_halo_invariance() {
  const int64_t nx = 29, ny = 31;
  // Reference: 12 single steps on a halo-1 layout.
  auto run = [&](int halo, int steps) {
    Layout L = Layout::make(nx, ny, halo);
    std::vector<float> a(size_t(L.elems())), b(size_t(L.elems()));
    cpu::init_field(a.data() + L.origin(), L, 0, 0, nx, ny, 2, 3);
    cpu::init_field(b.data() + L.origin(), L, 0, 0, nx, ny, 2, 3);
    cpu::Geom g;
    g.pitch = L.pitch;
    g.nx = nx;
    g.ny = ny;
    float* s = a.data() + L.origin();
    float* d = b.data() + L.origin();
    for (int k = 0; k < steps; ++k) {
      cpu::step(s, d, g, Box{0, nx, 0, ny}, false);
      std::swap(s, d);
    }
    std::vector<float> out(size_t(nx * ny));
    for (int64_t r = 0; r < nx; ++r) std::memcpy(&out[size_t(r * ny)], s + r * L.pitch, size_t(ny) * 4);
    return out;
  };
  auto x = run(1, 12), y = run(4, 12);
  EXPECT(x == y);
  // boundary ring unchanged
  EXPECT(x[0] == init_random(0, 0, 3) && x[size_t(nx * ny - 1)] == init_random(nx - 1, ny - 1, 3));
}

int main() {
  test_dims();
  test_blocks();
  test_format();
  test_init_wrap();
  test_cpu_step_and_halo_invariance();
  if (failures) {
    std::fprintf(stderr, "selftest: %d failure(s)\n", failures);
    return 1;
  }
  std::printf("selftest: ok\n");
  return 0;
}
