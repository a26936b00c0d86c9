// Grid I/O.
//
// * Text ".dat" output byte-compatible with the reference's prtdat
//   (cuda/cuda_heat.cu:285-300, mpi/mpi_heat_improved_persistent_stat.c:326-341):
//   "%6.1f" values, one line per iy from ny-1 down to 0 (transposed and
//   y-flipped), ix left to right, single spaces, '\n' at line end.
// * A reader for that format (tests, round trips).
// * A raw binary format with a small header, used for output of grids too
//   large for text and for checkpoint/resume (the reference has neither).
// * An order-independent checksum so huge runs can be compared across
//   decompositions without moving the grid to one host.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace heat {

// Append the "%6.1f" rendering of v to out (bit-exact with glibc printf).
void format_6_1f(float v, std::string& out);

// Write a full nx x ny row-major grid in prtdat format.
void write_dat(const std::string& path, int64_t nx, int64_t ny, const float* grid);
// Read a prtdat file back into an nx x ny row-major grid (values are the
// printed, i.e. rounded, numbers).
std::vector<float> read_dat(const std::string& path, int64_t* nx, int64_t* ny);

struct BinHeader {
  char magic[8];       // "HEATF32\0"
  uint32_t version;    // 1
  uint32_t parity;     // reserved (buffer parity at checkpoint time)
  int64_t nx, ny;
  int64_t step;        // completed steps
  float cx, cy;
  uint64_t reserved[3];  // [0]: bin_config_tag of the writer (0 = unknown)
};
static_assert(sizeof(BinHeader) == 72, "BinHeader layout");

// Create/truncate a binary grid file and write its header (rank 0).
void bin_create(const std::string& path, const BinHeader& h);
// Write a block of rows [ox, ox+lx) x cols [oy, oy+ly) taken from a strided
// source into an existing binary grid file (every rank writes its own block).
void bin_write_block(const std::string& path, int64_t nx, int64_t ny, int64_t ox, int64_t oy,
                     int64_t lx, int64_t ly, const float* src, int64_t src_pitch);
BinHeader bin_read_header(const std::string& path);
// fsync `tmp` and rename it over `path` (atomic replacement of a checkpoint).
void bin_commit(const std::string& tmp, const std::string& path);
// Header tag of the modes that change the continuation of a run.
inline uint64_t bin_config_tag(int compat, int numerics) {
  return (uint64_t(1) << 63) | (uint64_t(numerics & 0xff) << 8) | uint64_t(compat & 0xff);
}
void bin_read_block(const std::string& path, int64_t ox, int64_t oy, int64_t lx, int64_t ly,
                    float* dst, int64_t dst_pitch);

// Order-independent checksum of a block of cells with their global indices.
struct Checksum {
  uint64_t hash = 0;   // sum mod 2^64 of mix(bits, global index): order independent
  double sum = 0.0;    // plain fp64 sum (order dependent in the last bits)
  double min = 0.0, max = 0.0;
  int64_t count = 0;
  void merge(const Checksum& o);
};
Checksum checksum_block(const float* src, int64_t src_pitch, int64_t ox, int64_t oy, int64_t lx,
                        int64_t ly, int64_t ny);

}  // namespace heat
