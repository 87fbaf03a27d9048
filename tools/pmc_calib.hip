// FETCH_SIZE / WRITE_SIZE calibration for the access widths the Canny front
// end uses (MI355X_MICROARCH.md: only 16-B-per-lane streams are calibrated):
// a 1 GiB buffer read once with 12-byte-per-lane loads (three dwords, stride
// 12 B: k_canny's BGR groups), once with 16-byte loads, and 4-byte-per-lane
// stores of 16 B per 128-px tile row (k_canny's bit-plane words); round 5:
// 4-byte-per-lane coalesced loads and stores (bit-plane rows) and 2^24
// unaligned 4-byte gathers at random offsets (the scorers' pixel loads).
// Run: rocprofv3 --kernel-trace --pmc FETCH_SIZE -- ./pmc_calib (and WRITE_SIZE).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void rd12(const uint32_t* __restrict__ p, size_t n3, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n3; i += (size_t)gridDim.x * blockDim.x) {
    const uint32_t* q = p + 3 * i;
    acc ^= q[0] + q[1] * 3u + q[2] * 7u;
  }
  if (acc == 0x12345678u) out[0] = acc;
}
__global__ void rd16(const uint4* __restrict__ p, size_t n4, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    acc ^= v.x + v.y * 3u + v.z * 5u + v.w * 7u;
  }
  if (acc == 0x12345678u) out[0] = acc;
}
// one 64-thread group per 16-row x 4-word tile of a row-major plane with WW words per row
__global__ void wr_tiles(uint32_t* __restrict__ plane, int WW, int H) {
  const int tx = blockIdx.x, ty = blockIdx.y, t = threadIdx.x;
  const int y = ty * 16 + (t >> 2), w = tx * 4 + (t & 3);
  if (y < H && w < WW) plane[(size_t)blockIdx.z * WW * H + (size_t)y * WW + w] = 0x5a5a5a5au ^ (uint32_t)(y * w);
}
// 4 bytes per lane, consecutive lanes consecutive dwords (the bit-plane row
// loads / stores of k_hyst_rec, k_morph_walk, k_canny_strip's plane words)
__global__ void rd4(const uint32_t* __restrict__ p, size_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc ^= p[i] * 3u;
  if (acc == 0x12345678u) out[0] = acc;
}
__global__ void wr4(uint32_t* __restrict__ p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = (uint32_t)i * 0x9e3779b9u;
}
// unaligned dword gathers at pseudo-random byte offsets of a 1 GiB buffer (the
// scorers' pixel loads): one 4-byte load per lane, 2^24 of them
__global__ void rdgather(const uint8_t* __restrict__ p, size_t bytes, uint32_t* out) {
  typedef __attribute__((aligned(1))) const uint32_t u32u;
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < ((size_t)1 << 24); i += (size_t)gridDim.x * blockDim.x) {
    const size_t off = ((i * 0x9e3779b97f4a7c15ull) >> 20) % (bytes - 4);
    acc ^= *(u32u*)(p + off);
  }
  if (acc == 0x12345678u) out[0] = acc;
}
int main() {
  const size_t bytes = (size_t)1 << 30;
  uint32_t *buf, *out;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  (void)hipMemset(buf, 1, bytes);
  rd12<<<4096, 256>>>(buf, bytes / 12, out);
  rd16<<<4096, 256>>>((const uint4*)buf, bytes / 16, out);
  const int WW = 40, H = 720, F = 4096;  // 1280x720 bit planes, 4096 frames = 472 MB
  wr_tiles<<<dim3(10, 45, F), 64>>>(buf, WW, H);
  rd4<<<4096, 256>>>(buf, bytes / 4, out);
  wr4<<<4096, 256>>>(buf, bytes / 4);
  rdgather<<<4096, 256>>>((const uint8_t*)buf, bytes, out);
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  printf("read bytes per kernel %zu (rd12 %zu); tile-word write bytes %zu; rd4 / wr4 bytes %zu; rdgather loads %d x 4 B\n",
         bytes, (bytes / 12) * 12, (size_t)WW * H * F * 4, bytes, 1 << 24);
  return 0;
}
