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
  auto load8 = [&](int32_t j) -> uint64_t {
    uint64_t w = 0;
    for (int b = 0; b < 8 && 8 * j + b < n; b++) w |= (uint64_t)s[8 * j + b] << (8 * b);
    return w;
  };
  return dk::simple_path_hash(n, load8, seed, h) ? 1 : 0;
}
extern "C" int prod_simple8(uint64_t w) { return dk::simple8(w) ? 1 : 0; }
extern "C" int prod_uri_class_simple(uint32_t c) { return (dk::uri_class((uint8_t)c) & dk::CC_SIMPLE) ? 1 : 0; }
