// A one-kernel device code object for the host-only ASan build (tests/asan/Makefile): the host-only
// objects reference one fatbin symbol per translation unit; each is bound to this bundle so the
// runtime's static registration sees a well-formed (empty of our kernels) code object.  No kernel of
// the library can launch from that build -- it only checks host code.
#include <hip/hip_runtime.h>
__global__ void iwq_asan_placeholder(int* p) {
  if (p) p[0] = 1;
}
