// Host build of the HTTP slow path's executor (cilium_amd/csrc/regex_vm.h)
// for the program interpreter (tests/program_interp.py).  Test infrastructure.
#include <cstdint>
#include <vector>

#include "../../cilium_amd/csrc/regex_vm.h"

extern "C" int vm_host_match(const uint32_t* prog, const uint8_t* s, uint32_t n, uint32_t scratch_words,
                             uint32_t max_steps) {
  thread_local std::vector<uint32_t> scratch;
  if (scratch.size() < scratch_words) scratch.resize(scratch_words);
  return l7m::vm_match(prog, s, n, scratch.data(), scratch_words, max_steps);
}
