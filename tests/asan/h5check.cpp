// Host-only driver of the HDF5 reader (csrc/h5read.cpp) for the AddressSanitizer
// build (`make asan` -> build/asan/h5check): reads one dataset of a file the way
// dataset.read_h5 does (pcadv_h5_info, then pcadv_h5_read as f32 and as int64,
// whole and with a first-dimension cut) and prints what it got or the error.
//   h5check <file> <dataset> [keep1]
// Exit status 0 = read, 1 = a clean error from the reader; anything else (a
// sanitizer report, a signal) is a bug.  Test infrastructure only.
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "pcadv.h"

namespace pcadv {
static char g_err[512];
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
}
}  // namespace pcadv

extern "C" const char* pcadv_last_error(void) { return pcadv::g_err; }

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: h5check <file> <dataset> [keep1]\n");
    return 2;
  }
  const int64_t keep1 = argc > 3 ? std::atoll(argv[3]) : 0;
  int rank = 0, dt = 0;
  int64_t dims[8] = {0};
  if (pcadv_h5_info(argv[1], argv[2], &rank, dims, &dt) != 0) {
    std::printf("error: %s\n", pcadv_last_error());
    return 1;
  }
  int64_t n = 1;
  for (int i = 0; i < rank; ++i) {
    const int64_t d = (i == 1 && keep1 > 0 && keep1 < dims[1]) ? keep1 : dims[i];
    if (d < 0 || (d > 0 && n > (int64_t(1) << 28) / d)) {  // the caller's size guard
      std::printf("error: dataset too large for the driver\n");
      return 1;
    }
    n *= d;
  }
  std::vector<float> f(n > 0 ? n : 1);
  std::vector<int64_t> q(n > 0 ? n : 1);
  int rc = pcadv_h5_read(argv[1], argv[2], 0, keep1, f.data(), n * sizeof(float));
  if (rc == 0) rc = pcadv_h5_read(argv[1], argv[2], 1, keep1, q.data(), n * sizeof(int64_t));
  if (rc != 0) {
    std::printf("error: %s\n", pcadv_last_error());
    return 1;
  }
  double s = 0;
  for (int64_t i = 0; i < n; ++i) s += f[i];
  std::printf("ok rank=%d n=%lld sum=%g\n", rank, (long long)n, s);
  return 0;
}
