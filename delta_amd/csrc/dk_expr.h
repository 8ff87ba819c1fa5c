// Compiled predicate programs (dk_program, include/dkgpu.h), shared by the compiler (dk_expr.cpp) and
// the host code that installs and runs them (dk_host.cpp). Host memory only; dk_host.cpp lays a
// program out in one device buffer (DSkipProg / DPartProg, dk_device.h) when it is installed.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

struct dk_program {
  int32_t kind = 0;                            // DK_PROGRAM_SKIPPING (0) / DK_PROGRAM_PARTITION (1)
  // data skipping: the stats fields read from each row's stats (type code SK_*, name components)
  std::vector<int32_t> path_type;
  std::vector<std::vector<std::string>> paths;
  // partition pruning: the partition columns (type code PT_*, physical name)
  std::vector<int32_t> field_type;
  std::vector<std::string> fields;
  // postfix program and its pool (field / path names first, then literal bytes)
  std::vector<int32_t> op, arg;
  std::vector<int64_t> lit;
  std::string pool;
  std::vector<int32_t> comp_off, comp_len, path_comp;   // skipping: name components in pool
  std::vector<int32_t> name_off, name_len;              // partition: field names in pool
  int32_t stack = 0;                           // deepest evaluation stack
};

namespace dk {
int dk_fail(const std::string& m);             // sets the thread's dk_last_error (dk_host.cpp)
// the byte image of a program's device layout: int32 / int64 arrays and the pool, 8-byte aligned;
// offs[] receives each array's byte offset (skipping: path_type, path_comp, comp_off, comp_len, op,
// arg, lit, pool; partition: field_type, name_off, name_len, op, arg, lit, pool)
std::string program_image(const dk_program& p, int64_t offs[8]);
}  // namespace dk
