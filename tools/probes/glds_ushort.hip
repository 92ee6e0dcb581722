// Probe: LDS layout written by global_load_lds_ushort (2-byte LDS-DMA) on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void k(const uint16_t* g, uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint32_t smem[256];
  for (int i = threadIdx.x; i < 256; i += 64) smem[i] = 0xDEADBEEFu;
  __syncthreads();
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(g + threadIdx.x),
                                   (__attribute__((address_space(3))) void*)((uint8_t*)smem), 2, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 256; i += 64) out[i] = smem[i];
}
int main() {
  uint16_t h[64];
  for (int i = 0; i < 64; ++i) h[i] = (uint16_t)(0x1000 + i);
  uint16_t* dg; uint32_t* dout;
  hipMalloc(&dg, sizeof h); hipMalloc(&dout, 1024);
  hipMemcpy(dg, h, sizeof h, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dg, dout);
  uint32_t o[256];
  hipMemcpy(o, dout, 1024, hipMemcpyDeviceToHost);
  for (int i = 0; i < 40; ++i) printf("%08x%c", o[i], (i % 8 == 7) ? '\n' : ' ');
  return 0;
}
