// io.cpp -- the on-disk point format of the reference's ModelNet40 loader
// (SURVEY.md 8f row f3): modelnet40_normal_resampled/<class>/<name>.txt holds
// one point per line, "x,y,z,nx,ny,nz".  The reference parses it with
// np.loadtxt(delimiter=',') into float64 and casts to float32
// (datasets/modelnet40.py:30, :44-45).  This parser does the same per value
// (strtod, then a cast to float), so it gives the same bits, and it is native:
// one pass over an in-memory copy of the file, no Python per line.  Host code
// only; the caller copies the rows to the device.
#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "common.hpp"

namespace pcr {
namespace {

bool read_file(const char* path, std::vector<char>* buf) {
  FILE* f = fopen(path, "rb");
  if (!f) return false;
  buf->clear();
  char chunk[1 << 16];
  size_t got;
  while ((got = fread(chunk, 1, sizeof(chunk), f)) > 0) buf->insert(buf->end(), chunk, chunk + got);
  fclose(f);
  buf->push_back('\0');
  return true;
}

inline bool is_blank(char c) { return c == ' ' || c == '\t' || c == '\r'; }

// Parses the rows; out == nullptr only counts.  Returns rows, or -1 with an
// error set (ragged rows, junk, missing file).
long long parse_rows(const char* path, int* cols_io, float* out, long long max_rows) {
  std::vector<char> buf;
  if (!read_file(path, &buf)) {
    set_error("read_xyzn_txt: cannot open %s (%s)", path, strerror(errno));
    return -1;
  }
  const char* p = buf.data();
  long long rows = 0;
  int cols = *cols_io;
  while (*p) {
    while (is_blank(*p)) p++;
    if (*p == '\n') {  // blank line (np.loadtxt skips it)
      p++;
      continue;
    }
    if (!*p) break;
    int c = 0;
    for (;;) {
      char* end;
      const double v = strtod(p, &end);
      if (end == p) {
        set_error("read_xyzn_txt: %s: row %lld: not a number", path, rows + 1);
        return -1;
      }
      if (out) {
        if (rows >= max_rows || c >= cols) {
          set_error("read_xyzn_txt: %s: more data than the %lld x %d buffer", path, max_rows,
                    cols);
          return -1;
        }
        out[rows * cols + c] = (float)v;
      }
      c++;
      p = end;
      while (is_blank(*p)) p++;
      if (*p == ',') {
        p++;
        continue;
      }
      break;
    }
    if (*p && *p != '\n') {
      set_error("read_xyzn_txt: %s: row %lld: unexpected character", path, rows + 1);
      return -1;
    }
    if (*p == '\n') p++;
    if (cols <= 0) cols = c;
    if (c != cols) {
      set_error("read_xyzn_txt: %s: row %lld has %d columns, expected %d", path, rows + 1, c,
                cols);
      return -1;
    }
    rows++;
  }
  *cols_io = cols;
  return rows;
}

}  // namespace
}  // namespace pcr

using namespace pcr;

extern "C" pcr_status pcr_txt_shape(const char* path, long long* rows, int* cols) {
  PCR_REQUIRE(path && rows && cols, "txt_shape: null argument");
  int c = 0;
  const long long r = parse_rows(path, &c, nullptr, 0);
  if (r < 0) return PCR_ERR_INVALID;
  *rows = r;
  *cols = c;
  return PCR_OK;
}

extern "C" pcr_status pcr_read_xyzn_txt(const char* path, float* out, long long rows, int cols) {
  PCR_REQUIRE(path && out && rows >= 0 && cols >= 1, "read_xyzn_txt: invalid arguments");
  int c = cols;
  const long long r = parse_rows(path, &c, out, rows);
  if (r < 0) return PCR_ERR_INVALID;
  PCR_REQUIRE(r == rows, "read_xyzn_txt: %s has %lld rows, buffer %lld", path, r, rows);
  return PCR_OK;
}
