// Streaming-read probe (GPU box): the strip Canny's BGR access geometry --
// one wave walks the rows of a 480-column strip of a 1280x720 BGR frame, 24 B
// per lane per row (two 12-byte loads, lanes 24 B apart) -- against wider
// loads and deeper row prefetch, over 4096 frames (11.3 GB, past every cache).
// Prints GB/s per variant. Usage: ./stream_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int W = 1280, H = 720, F = 4096, STRIPS = 3, RSTEP = 3 * W;
typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// MODE 0: 2 x dwordx3 per lane (24 B, the strip kernel); MODE 1: 1 x dwordx4 + 1 x dwordx2 per lane (24 B);
// MODE 2: lanes 16 B apart, 1.5 KB per row as 1 x dwordx4 (lanes 0..63) + 1 x dwordx2 (lanes 0..63)
template <int MODE, int DEPTH>
__global__ __launch_bounds__(256) void probe(const uint8_t* __restrict__ bgr, uint32_t* out) {
  const int gw = (blockIdx.x * 256 + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  if (gw >= F * STRIPS) return;
  const int f = gw / STRIPS, s = gw % STRIPS;
  const uint8_t* base = bgr + (size_t)f * RSTEP * H + (size_t)s * 480 * 3;
  uint32_t acc = 0;
  uint32_t q[DEPTH][6];
  auto ld = [&](int row, uint32_t* d) {
    const uint8_t* p = base + (size_t)row * RSTEP;
    if (MODE == 0) {
      const u32x3 a = *(const u32x3*)(p + lane * 24), b = *(const u32x3*)(p + lane * 24 + 12);
      d[0] = a.x; d[1] = a.y; d[2] = a.z; d[3] = b.x; d[4] = b.y; d[5] = b.z;
    } else if (MODE == 1) {
      const u32x4 a = *(const u32x4*)(p + lane * 24);
      const uint2 b = *(const uint2*)(p + lane * 24 + 16);
      d[0] = a.x; d[1] = a.y; d[2] = a.z; d[3] = a.w; d[4] = b.x; d[5] = b.y;
    } else {
      const u32x4 a = *(const u32x4*)(p + lane * 16);
      const uint2 b = *(const uint2*)(p + 1024 + lane * 8);
      d[0] = a.x; d[1] = a.y; d[2] = a.z; d[3] = a.w; d[4] = b.x; d[5] = b.y;
    }
  };
#pragma unroll
  for (int k = 0; k < DEPTH; k++) ld(k, q[k]);
  for (int r = 0; r < H; r += DEPTH) {
#pragma unroll
    for (int k = 0; k < DEPTH; k++) {
#pragma unroll
      for (int j = 0; j < 6; j++) acc = acc * 31u + q[k][j];
      // some ALU per row, like a stencil step (~100 instructions)
#pragma unroll 1
      for (int z = 0; z < 8; z++) acc = (acc ^ (acc >> 7)) * 0x9E3779B1u + (uint32_t)z;
      const int nr = r + k + DEPTH;
      ld(nr < H ? nr : H - 1, q[k]);
    }
  }
  if (acc == 0x12345678u) out[gw * 64 + lane] = acc;  // keep the loads
}

template <int MODE, int DEPTH>
void run(const uint8_t* d, uint32_t* o, const char* name) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int blocks = (F * STRIPS * 64 + 255) / 256;
  probe<MODE, DEPTH><<<blocks, 256>>>(d, o);
  hipEventRecord(a);
  for (int it = 0; it < 3; it++) probe<MODE, DEPTH><<<blocks, 256>>>(d, o);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  ms /= 3;
  const double bytes = (double)F * STRIPS * H * 64 * 24;
  printf("%-28s %8.3f ms  %8.1f GB/s\n", name, ms, bytes / ms / 1e6);
}

int main() {
  uint8_t* d;
  uint32_t* o;
  const size_t n = (size_t)F * RSTEP * H + 4096;
  if (hipMalloc(&d, n) != hipSuccess || hipMalloc(&o, (size_t)F * STRIPS * 64 * 4) != hipSuccess) return 1;
  hipMemset(d, 7, n);
  hipDeviceSynchronize();
  run<0, 1>(d, o, "2x dwordx3, depth 1");
  run<0, 2>(d, o, "2x dwordx3, depth 2");
  run<0, 4>(d, o, "2x dwordx3, depth 4");
  run<1, 1>(d, o, "dwordx4+x2, depth 1");
  run<1, 2>(d, o, "dwordx4+x2, depth 2");
  run<2, 1>(d, o, "contig x4+x2, depth 1");
  run<2, 2>(d, o, "contig x4+x2, depth 2");
  run<2, 4>(d, o, "contig x4+x2, depth 4");
  return 0;
}
