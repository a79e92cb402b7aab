// tools/ipc_probe.hip -- does a peer-mapped exchange work between processes on this box?
//
// usage: ipc_probe <rank> <world> <dir> <alloc: 0 hipMalloc | 1 fine-grained | 3 uncached>
// Each process allocates a receive region + flags with the given allocation kind, writes its
// IPC handle to <dir>/h<rank>, opens every peer's handle, then one kernel stores a rank pattern
// into every peer's slot and signals the peer's flag; a second kernel waits (bounded, 10 s) for
// every peer's flag; the host checks the slots.  Prints one line: OK or what failed.
// (Diagnostic for the PeerComm design, host/comm.cpp; processes on one GPU or on several.)
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::printf("FAIL %s: %s\n", #x, hipGetErrorString(e_));                  \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

constexpr int kSlot = 1 << 16;  // floats per slot

struct Peers {
  float *recv[8];
  unsigned *flags[8];
};

__global__ void k_push(Peers p, int rank, int world, unsigned gen) {
  for (int q = 0; q < world; q++) {
    float *dst = p.recv[q] + (size_t)rank * kSlot;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < kSlot; i += gridDim.x * blockDim.x)
      dst[i] = (float)(rank * 1000003 + i);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    // (one block: its stores are done; the flag after them)
    for (int q = 0; q < world; q++)
      __hip_atomic_store(p.flags[q] + rank, gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ void k_wait(unsigned *flags, int world, unsigned gen, unsigned *err) {
  const int q = threadIdx.x;
  if (q >= world) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while ((int)(__hip_atomic_load(flags + q, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - gen) < 0) {
    __builtin_amdgcn_s_sleep(10);
    if (__builtin_amdgcn_s_memrealtime() - t0 > 1000000000ull) {  // 10 s at 100 MHz
      __hip_atomic_store(err, 1u + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
  }
}

int main(int argc, char **argv) {
  if (argc < 5) return 2;
  const int rank = std::atoi(argv[1]), world = std::atoi(argv[2]), kind = std::atoi(argv[4]);
  const std::string dir = argv[3];
  int ndev = 0;
  CK(hipGetDeviceCount(&ndev));
  CK(hipSetDevice(rank % ndev));
  const size_t bytes = (size_t)world * kSlot * 4 + 4096;
  void *base = nullptr;
  if (kind == 0)
    CK(hipMalloc(&base, bytes));
  else
    CK(hipExtMallocWithFlags(&base, bytes, (unsigned)kind));
  CK(hipMemset(base, 0, bytes));
  CK(hipDeviceSynchronize());
  hipIpcMemHandle_t h;
  CK(hipIpcGetMemHandle(&h, base));
  {
    std::ofstream f(dir + "/h" + std::to_string(rank) + ".tmp", std::ios::binary);
    f.write(reinterpret_cast<const char *>(&h), sizeof h);
  }
  std::rename((dir + "/h" + std::to_string(rank) + ".tmp").c_str(),
              (dir + "/h" + std::to_string(rank)).c_str());
  Peers p{};
  for (int q = 0; q < world; q++) {
    void *ptr = base;
    if (q != rank) {
      hipIpcMemHandle_t hq;
      const std::string fn = dir + "/h" + std::to_string(q);
      for (int t = 0;; t++) {
        std::ifstream f(fn, std::ios::binary);
        if (f.read(reinterpret_cast<char *>(&hq), sizeof hq)) break;
        if (t > 600) {
          std::printf("FAIL rank %d: no handle from %d\n", rank, q);
          return 1;
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(100));
      }
      CK(hipIpcOpenMemHandle(&ptr, hq, hipIpcMemLazyEnablePeerAccess));
    }
    p.recv[q] = static_cast<float *>(ptr);
    p.flags[q] = reinterpret_cast<unsigned *>(static_cast<char *>(ptr) + (size_t)world * kSlot * 4);
  }
  unsigned *err = nullptr;
  CK(hipMalloc(&err, 4));
  CK(hipMemset(err, 0, 4));
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned gen = 1; gen <= 3; gen++) {
    k_push<<<64, 256>>>(p, rank, world, gen);
    k_wait<<<1, 64>>>(p.flags[rank], world, gen, err);
  }
  CK(hipDeviceSynchronize());
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  unsigned e = 0;
  CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
  if (e) {
    std::printf("FAIL rank %d: timeout waiting for rank %u\n", rank, e - 1);
    return 1;
  }
  std::vector<float> got((size_t)world * kSlot);
  CK(hipMemcpy(got.data(), base, got.size() * 4, hipMemcpyDeviceToHost));
  long bad = 0;
  for (int q = 0; q < world; q++)
    for (int i = 0; i < kSlot; i++) bad += got[(size_t)q * kSlot + i] != (float)(q * 1000003 + i);
  std::printf("%s rank %d world %d kind %d devices %d: %ld bad, %.2f ms\n", bad ? "FAIL" : "OK",
              rank, world, kind, ndev, bad, ms);
  // every process done before anyone frees (peers may still be checking)
  {
    std::ofstream f(dir + "/d" + std::to_string(rank));
    f << 1;
  }
  for (int q = 0; q < world; q++)
    for (int t = 0; t < 600; t++) {
      std::ifstream f(dir + "/d" + std::to_string(q));
      if (f.good()) break;
      std::this_thread::sleep_for(std::chrono::milliseconds(50));
    }
  for (int q = 0; q < world; q++)
    if (q != rank) CK(hipIpcCloseMemHandle(p.recv[q]));
  CK(hipFree(base));
  return bad ? 1 : 0;
}
