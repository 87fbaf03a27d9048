// v_perm_b32 sign selectors (8..11 replicate a sign bit) against the
// two-shift sign_pair of kernels.hip, on 2^24 random operand pairs.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
__global__ void k(uint32_t* bad, uint32_t sel) {
  uint32_t st = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t nbad = 0;
  for (int it = 0; it < 16; it++) {
    st = st * 1664525u + 1013904223u;
    const int32_t lo = (int32_t)st;
    st = st * 1664525u + 1013904223u;
    const int32_t hi = (int32_t)st;
    const uint32_t ref = __builtin_amdgcn_perm((uint32_t)(hi >> 31), (uint32_t)(lo >> 31), 0x05040100u);
    const uint32_t got = __builtin_amdgcn_perm((uint32_t)hi, (uint32_t)lo, sel);
    nbad += ref != got;
  }
  if (nbad) atomicAdd(bad, nbad);
}
int main() {
  uint32_t* d;
  (void)hipMalloc(&d, 4);
  const uint32_t sels[] = {0x0B0B0909u, 0x09090B0Bu, 0x0A0A0808u, 0x08080A0Au};
  for (uint32_t s : sels) {
    (void)hipMemset(d, 0, 4);
    k<<<4096, 256>>>(d, s);
    uint32_t h = 0;
    (void)hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
    printf("sel %08x: %u mismatches of %u\n", s, h, 4096u * 256u * 16u);
  }
  return 0;
}
