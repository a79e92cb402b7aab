// tools/ta_micro.hip -- vector-memory issue-cost microbenchmark for gfx950 (diagnostic tool).
// Measures, for an L2-resident table, how the cost of a wave-wide load depends on the
// access width and on how many distinct rows / lines one instruction touches.  Used to pick
// the GraphSum lane mapping.  Build: hipcc -O3 --offload-arch=gfx950 tools/ta_micro.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);         \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

constexpr int TABLE_ROWS = 16384;  // x 64 B = 1 MB (L2 resident)
constexpr int ITERS = 4096;

// MODE 0: float4, 16 rows x 64 B per instruction (GraphSum d=16 gather shape)
// MODE 1: float4, 64 rows x 16 B per instruction (one lane per row)
// MODE 2: float4, fully contiguous 1 KB per instruction
// MODE 3: dword, 64 distinct contiguous (256 B)
// MODE 4: dword, 16 distinct, each replicated in 4 lanes (GraphSum idx loads)
// MODE 5: float2, 32 rows x ... (8 B lanes, 8 lanes per 64-B row)
// MODE 6: dword via scalar-uniform address (all lanes same)
template <int MODE>
__global__ __launch_bounds__(256) void k(const float4 *__restrict__ table, float4 *out, int salt) {
  const int lane = threadIdx.x & 63;
  unsigned h = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 2654435761u + salt;
  float4 acc = make_float4(0, 0, 0, 0);
  const float *tf = reinterpret_cast<const float *>(table);
  const float2 *t2 = reinterpret_cast<const float2 *>(table);
#pragma unroll 4
  for (int it = 0; it < ITERS; it++) {
    h = h * 1664525u + 1013904223u;
    unsigned r = h >> 8;
    if (MODE == 0) {
      const int row = (r + (lane >> 2) * 977) & (TABLE_ROWS - 1);
      const float4 x = table[row * 4 + (lane & 3)];
      acc.x += x.x; acc.y += x.y; acc.z += x.z; acc.w += x.w;
    } else if (MODE == 1) {
      const int row = (r + lane * 977) & (TABLE_ROWS - 1);
      const float4 x = table[row * 4];
      acc.x += x.x; acc.y += x.y; acc.z += x.z; acc.w += x.w;
    } else if (MODE == 2) {
      const int base = (r & (TABLE_ROWS * 4 - 1)) & ~63;
      const float4 x = table[base + lane];
      acc.x += x.x; acc.y += x.y; acc.z += x.z; acc.w += x.w;
    } else if (MODE == 3) {
      const int base = (r & (TABLE_ROWS * 16 - 1)) & ~63;
      acc.x += tf[base + lane];
    } else if (MODE == 4) {
      const int base = (r & (TABLE_ROWS * 16 - 1)) & ~63;
      acc.x += tf[base + (lane >> 2)];
    } else if (MODE == 5) {
      const int row = (r + (lane >> 3) * 977) & (TABLE_ROWS - 1);
      const float2 x = t2[row * 8 + (lane & 7)];
      acc.x += x.x; acc.y += x.y;
    } else if (MODE == 6) {
      const int base = r & (TABLE_ROWS * 16 - 1);
      acc.x += tf[base];
    }
  }
  if (acc.x == 12345.678f) out[0] = acc;
}

template <int MODE>
double run(const float4 *t, float4 *o, int blocks) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, t, o, 1);
  CHECK(hipEventRecord(a));
  for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, t, o, r);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / 5;
}

int main() {
  float4 *t, *o;
  CHECK(hipMalloc(&t, (size_t)TABLE_ROWS * 64));
  CHECK(hipMemset(t, 0, (size_t)TABLE_ROWS * 64));
  CHECK(hipMalloc(&o, 64));
  const int blocks = 256 * 8;  // 8 WGs of 4 waves per CU
  const double insts = (double)blocks * 4 * ITERS;  // wave-level load instructions
  const char *names[] = {"f4 16rows x64B", "f4 64rows x16B", "f4 contiguous 1KB", "dword 64 distinct",
                         "dword 16 distinct x4", "f2 8rows x64B", "dword uniform"};
  const double bytes[] = {1024, 1024, 1024, 256, 256, 512, 256};
  double ms[7];
  ms[0] = run<0>(t, o, blocks);
  ms[1] = run<1>(t, o, blocks);
  ms[2] = run<2>(t, o, blocks);
  ms[3] = run<3>(t, o, blocks);
  ms[4] = run<4>(t, o, blocks);
  ms[5] = run<5>(t, o, blocks);
  ms[6] = run<6>(t, o, blocks);
  printf("{");
  for (int m = 0; m < 7; m++) {
    const double cyc = ms[m] * 1e-3 * 2.4e9 * 256 / insts;  // CU-cycles per wave instruction
    printf("\"%s\": {\"ms\": %.3f, \"cu_cycles_per_inst\": %.2f, \"lane_bytes_TBs\": %.2f}%s",
           names[m], ms[m], cyc, insts * bytes[m] / (ms[m] * 1e-3) / 1e12, m < 6 ? ", " : "");
  }
  printf("}\n");
  return 0;
}
