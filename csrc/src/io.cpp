// Grid I/O: prtdat-compatible text, binary blocks, checksums.
#include "heat/io.hpp"

#include <fcntl.h>
#include <unistd.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <limits>

#include "heat/common.hpp"
#include "heat/init_fn.hpp"

namespace heat {

void format_6_1f(float v, std::string& out) {
  // v*10 is exact in double for every finite float (24 + 4 mantissa bits), so
  // rounding it with the current (nearest-even) mode reproduces printf's
  // correctly rounded "%.1f" exactly, ties included.
  if (!std::isfinite(v) || std::fabs(v) >= 1e15f) {
    char buf[64];
    int n = std::snprintf(buf, sizeof buf, "%6.1f", double(v));
    out.append(buf, size_t(n));
    return;
  }
  double q = std::nearbyint(double(v) * 10.0);
  bool neg = std::signbit(v);
  uint64_t m = uint64_t(std::fabs(q));
  char digits[24];
  int nd = 0;
  uint64_t ip = m / 10;
  digits[nd++] = char('0' + m % 10);
  digits[nd++] = '.';
  do {
    digits[nd++] = char('0' + ip % 10);
    ip /= 10;
  } while (ip);
  if (neg) digits[nd++] = '-';
  for (int pad = nd; pad < 6; ++pad) out.push_back(' ');
  for (int i = nd - 1; i >= 0; --i) out.push_back(digits[i]);
}

void write_dat(const std::string& path, int64_t nx, int64_t ny, const float* grid) {
  FILE* fp = std::fopen(path.c_str(), "w");
  HEAT_CHECK(fp != nullptr, "cannot open %s for writing", path.c_str());
  std::string line;
  line.reserve(size_t(nx) * 8 + 8);
  for (int64_t iy = ny - 1; iy >= 0; --iy) {
    line.clear();
    for (int64_t ix = 0; ix < nx; ++ix) {
      format_6_1f(grid[ix * ny + iy], line);
      line.push_back(ix != nx - 1 ? ' ' : '\n');
    }
    HEAT_CHECK(std::fwrite(line.data(), 1, line.size(), fp) == line.size(), "short write to %s",
               path.c_str());
  }
  HEAT_CHECK(std::fclose(fp) == 0, "close %s", path.c_str());
}

std::vector<float> read_dat(const std::string& path, int64_t* nx_out, int64_t* ny_out) {
  std::ifstream in(path);
  HEAT_CHECK(in.good(), "cannot open %s", path.c_str());
  std::vector<std::vector<float>> lines;
  std::string line;
  while (std::getline(in, line)) {
    if (line.empty()) continue;
    std::vector<float> vals;
    const char* p = line.c_str();
    char* end = nullptr;
    while (true) {
      float v = std::strtof(p, &end);
      if (end == p) break;
      vals.push_back(v);
      p = end;
    }
    lines.push_back(std::move(vals));
  }
  const int64_t ny = int64_t(lines.size());
  HEAT_CHECK(ny > 0, "empty dat file %s", path.c_str());
  const int64_t nx = int64_t(lines[0].size());
  std::vector<float> g(size_t(nx * ny));
  for (int64_t l = 0; l < ny; ++l) {
    HEAT_CHECK(int64_t(lines[l].size()) == nx, "ragged dat file %s", path.c_str());
    const int64_t iy = ny - 1 - l;
    for (int64_t ix = 0; ix < nx; ++ix) g[ix * ny + iy] = lines[l][ix];
  }
  *nx_out = nx;
  *ny_out = ny;
  return g;
}

void bin_create(const std::string& path, const BinHeader& h) {
  int fd = ::open(path.c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0644);
  HEAT_CHECK(fd >= 0, "cannot create %s", path.c_str());
  HEAT_CHECK(::pwrite(fd, &h, sizeof h, 0) == ssize_t(sizeof h), "header write %s", path.c_str());
  // Size the file so every rank can pwrite its own block.
  const off_t total = off_t(sizeof h) + off_t(h.nx) * off_t(h.ny) * 4;
  HEAT_CHECK(::ftruncate(fd, total) == 0, "ftruncate %s", path.c_str());
  ::close(fd);
}

void bin_write_block(const std::string& path, int64_t nx, int64_t ny, int64_t ox, int64_t oy,
                     int64_t lx, int64_t ly, const float* src, int64_t src_pitch) {
  HEAT_CHECK(ox >= 0 && oy >= 0 && ox + lx <= nx && oy + ly <= ny, "block out of range");
  int fd = ::open(path.c_str(), O_WRONLY);
  HEAT_CHECK(fd >= 0, "cannot open %s", path.c_str());
  for (int64_t r = 0; r < lx; ++r) {
    const off_t off = off_t(sizeof(BinHeader)) + (off_t(ox + r) * ny + oy) * 4;
    const ssize_t n = ssize_t(ly * 4);
    HEAT_CHECK(::pwrite(fd, src + r * src_pitch, size_t(n), off) == n, "row write %s",
               path.c_str());
  }
  // Each rank makes its own rows durable before the commit barrier: ranks of
  // a TCP run may sit on different hosts, where rank 0's fsync does not
  // reach their page caches.
  const int rc = ::fsync(fd);
  ::close(fd);
  HEAT_CHECK(rc == 0, "fsync %s", path.c_str());
}

void bin_commit(const std::string& tmp, const std::string& path) {
  // Every rank has fsynced its rows (bin_write_block) and passed the caller's
  // barrier: fsync the header, rename, then fsync the directory so the swap
  // itself survives a crash (the previous checkpoint stays valid until then).
  int fd = ::open(tmp.c_str(), O_RDONLY);
  HEAT_CHECK(fd >= 0, "cannot open %s", tmp.c_str());
  const int rc = ::fsync(fd);
  ::close(fd);
  HEAT_CHECK(rc == 0, "fsync %s", tmp.c_str());
  HEAT_CHECK(::rename(tmp.c_str(), path.c_str()) == 0, "rename %s -> %s", tmp.c_str(),
             path.c_str());
  const size_t slash = path.find_last_of('/');
  const std::string dir = slash == std::string::npos ? "." : (slash == 0 ? "/" : path.substr(0, slash));
  const int dfd = ::open(dir.c_str(), O_RDONLY | O_DIRECTORY);
  HEAT_CHECK(dfd >= 0, "cannot open directory %s", dir.c_str());
  const int drc = ::fsync(dfd);
  ::close(dfd);
  HEAT_CHECK(drc == 0, "fsync directory %s", dir.c_str());
}

BinHeader bin_read_header(const std::string& path) {
  BinHeader h{};
  int fd = ::open(path.c_str(), O_RDONLY);
  HEAT_CHECK(fd >= 0, "cannot open %s", path.c_str());
  HEAT_CHECK(::pread(fd, &h, sizeof h, 0) == ssize_t(sizeof h), "header read %s", path.c_str());
  ::close(fd);
  HEAT_CHECK(std::memcmp(h.magic, "HEATF32", 8) == 0 && h.version == 1,
             "%s is not a heat binary grid", path.c_str());
  return h;
}

void bin_read_block(const std::string& path, int64_t ox, int64_t oy, int64_t lx, int64_t ly,
                    float* dst, int64_t dst_pitch) {
  BinHeader h = bin_read_header(path);
  HEAT_CHECK(ox >= 0 && oy >= 0 && ox + lx <= h.nx && oy + ly <= h.ny, "block out of range");
  int fd = ::open(path.c_str(), O_RDONLY);
  HEAT_CHECK(fd >= 0, "cannot open %s", path.c_str());
  for (int64_t r = 0; r < lx; ++r) {
    const off_t off = off_t(sizeof(BinHeader)) + (off_t(ox + r) * h.ny + oy) * 4;
    const ssize_t n = ssize_t(ly * 4);
    HEAT_CHECK(::pread(fd, dst + r * dst_pitch, size_t(n), off) == n, "row read %s",
               path.c_str());
  }
  ::close(fd);
}

void Checksum::merge(const Checksum& o) {
  if (o.count == 0) return;
  if (count == 0) {
    min = o.min;
    max = o.max;
  } else {
    min = std::min(min, o.min);
    max = std::max(max, o.max);
  }
  hash += o.hash;
  sum += o.sum;
  count += o.count;
}

Checksum checksum_block(const float* src, int64_t src_pitch, int64_t ox, int64_t oy, int64_t lx,
                        int64_t ly, int64_t ny) {
  Checksum c;
  c.min = std::numeric_limits<double>::infinity();
  c.max = -std::numeric_limits<double>::infinity();
  for (int64_t r = 0; r < lx; ++r) {
    const float* row = src + r * src_pitch;
    double rs = 0.0;
    for (int64_t j = 0; j < ly; ++j) {
      uint32_t bits;
      std::memcpy(&bits, &row[j], 4);
      const uint64_t gidx = uint64_t(ox + r) * uint64_t(ny) + uint64_t(oy + j);
      c.hash += mix64(gidx * 0x100000001B3ull ^ bits);
      const double v = row[j];
      rs += v;
      c.min = std::min(c.min, v);
      c.max = std::max(c.max, v);
    }
    c.sum += rs;
  }
  c.count = lx * ly;
  return c;
}

}  // namespace heat
