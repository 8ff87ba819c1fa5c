// CPU build of the product's host/device-shared key code (delta_amd/csrc/dk_uri.h) so the
// "not gpu" tests can check it against the oracle's java.net.URI restatement.
#include <stdint.h>
#include "../../delta_amd/csrc/dk_uri.h"

extern "C" int64_t prod_uri_canon(const uint8_t* s, int32_t n, uint8_t* out, int64_t cap) {
  dk::WriteSink w{out, 0, cap};
  int rc = dk::uri_emit(s, n, w);
  if (rc) return rc;
  return w.n;
}
extern "C" int prod_path_hash(const uint8_t* s, int32_t n, uint32_t seed, uint64_t* h) {
  return dk::path_hash(s, n, seed, h);
}
extern "C" int prod_simple_hash(const uint8_t* s, int32_t n, uint32_t seed, uint64_t* h) {
  dk::SimpleSet ss;
  auto load8 = [&](int32_t j) -> uint64_t {
    uint64_t w = 0;
    for (int b = 0; b < 8 && 8 * j + b < n; b++) w |= (uint64_t)s[8 * j + b] << (8 * b);
    return w;
  };
  return dk::simple_path_hash(n, load8, ss, seed, h) ? 1 : 0;
}
