// parallel-gcn_amd/csrc/host/comm.cpp
#include "comm.hpp"

#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>

#include "../common.hpp"
#include "../kernels.hpp"
#include "graph.hpp"

namespace pgcn {

int Partition::owner(int node) const {
  return (int)(std::upper_bound(bounds.begin(), bounds.end(), node) - bounds.begin()) - 1;
}

Partition make_partition(int n, const int *indptr, int world, int rank, int chunks) {
  PGCN_CHECK(world >= 1 && rank >= 0 && rank < world && n >= world, PGCN_E_INVALID,
             "partition: need 1 <= world <= n and 0 <= rank < world");
  PGCN_CHECK(chunks >= 1, PGCN_E_INVALID, "partition: chunks >= 1");
  Partition p;
  p.world = world;
  p.rank = rank;
  p.chunks = chunks;
  p.bounds.assign((size_t)world + 1, 0);
  p.bounds[(size_t)world] = n;
  const double total = (double)indptr[n];
  for (int r = 1; r < world; r++) {
    const double target = total * r / world;
    int lo = (int)(std::lower_bound(indptr, indptr + n + 1, (long long)target,
                                    [](int a, long long b) { return (long long)a < b; }) -
                   indptr);
    lo = std::max(lo, p.bounds[(size_t)r - 1] + 1);   // >= 1 node per rank
    lo = std::min(lo, n - (world - r));
    p.bounds[(size_t)r] = lo;
  }
  for (int r = 0; r < world; r++)
    p.maxrows = std::max(p.maxrows, p.bounds[(size_t)r + 1] - p.bounds[(size_t)r]);
  p.maxrows = (p.maxrows + chunks - 1) / chunks * chunks;
  return p;
}

void partition_subgraph_chunk(const Partition &part, int n, const int *indptr,
                              const int *indices, int k, std::vector<int> *sub_indptr,
                              std::vector<int> *sub_indices) {
  (void)n;
  const int lo = part.first(), hi = part.last(), W = part.world, h = part.chunk_rows();
  const long long rows = (long long)W * h;
  std::vector<int> cnt((size_t)rows, 0);
  auto node = [&](long long r) {  // chunk row -> global node (-1: padding)
    const int q = (int)(r / h), j = (int)(r % h);
    const int i = part.bounds[(size_t)q] + k * h + j;
    return i < part.bounds[(size_t)q + 1] ? i : -1;
  };
  parallel_for(rows, [&](long long b, long long e) {
    for (long long r = b; r < e; r++) {
      const int i = node(r);
      if (i < 0) continue;
      int c = 0;
      for (int t = indptr[i]; t < indptr[i + 1]; t++) c += (indices[t] >= lo && indices[t] < hi);
      cnt[(size_t)r] = c;
    }
  });
  sub_indptr->assign((size_t)rows + 1, 0);
  for (long long r = 0; r < rows; r++) (*sub_indptr)[(size_t)r + 1] = (*sub_indptr)[(size_t)r] + cnt[(size_t)r];
  sub_indices->assign((size_t)sub_indptr->back(), 0);
  parallel_for(rows, [&](long long b, long long e) {
    for (long long r = b; r < e; r++) {
      const int i = node(r);
      if (i < 0) continue;
      long long o = (*sub_indptr)[(size_t)r];
      for (int t = indptr[i]; t < indptr[i + 1]; t++) {
        const int j = indices[t];
        if (j >= lo && j < hi) (*sub_indices)[(size_t)o++] = j - lo;
      }
    }
  });
}

void partition_subgraph(const Partition &part, int n, const int *indptr, const int *indices,
                        std::vector<int> *sub_indptr, std::vector<int> *sub_indices,
                        std::vector<float> *sub_vals) {
  const int lo = part.first(), hi = part.last();
  const long long rows = (long long)part.world * part.maxrows;
  std::vector<int> cnt((size_t)rows, 0);
  auto padded = [&](int i) {
    const int q = part.owner(i);
    return (long long)q * part.maxrows + (i - part.bounds[(size_t)q]);
  };
  parallel_for(n, [&](long long b, long long e) {
    for (long long i = b; i < e; i++) {
      int c = 0;
      for (int k = indptr[i]; k < indptr[i + 1]; k++) c += (indices[k] >= lo && indices[k] < hi);
      cnt[(size_t)padded((int)i)] = c;
    }
  });
  sub_indptr->assign((size_t)rows + 1, 0);
  for (long long r = 0; r < rows; r++) (*sub_indptr)[(size_t)r + 1] = (*sub_indptr)[(size_t)r] + cnt[(size_t)r];
  sub_indices->assign((size_t)sub_indptr->back(), 0);
  sub_vals->assign((size_t)sub_indptr->back(), 0.0f);
  parallel_for(n, [&](long long b, long long e) {
    for (long long i = b; i < e; i++) {
      long long o = (*sub_indptr)[(size_t)padded((int)i)];
      const int di = indptr[i + 1] - indptr[i];
      for (int k = indptr[i]; k < indptr[i + 1]; k++) {
        const int j = indices[k];
        if (j >= lo && j < hi) {
          (*sub_indices)[(size_t)o] = j - lo;
          (*sub_vals)[(size_t)o] = graph_coef(di, indptr[j + 1] - indptr[j]);
          o++;
        }
      }
    }
  });
}

#define PGCN_NCCL(expr)                                                              \
  do {                                                                               \
    ncclResult_t r_ = (expr);                                                        \
    if (r_ != ncclSuccess)                                                           \
      throw Error(PGCN_E_COMM, std::string(#expr) + " -> " + ncclGetErrorString(r_)); \
  } while (0)

void Comm::unique_id(void *out128) {
  ncclUniqueId id;
  PGCN_NCCL(ncclGetUniqueId(&id));
  static_assert(sizeof(ncclUniqueId) == 128, "unexpected ncclUniqueId size");
  std::memcpy(out128, &id, sizeof id);
}

RcclComm::RcclComm(int rank, int world, const void *unique_id_128) : Comm(rank, world) {
  ncclUniqueId id;
  std::memcpy(&id, unique_id_128, sizeof id);
  ncclComm_t c;
  PGCN_NCCL(ncclCommInitRank(&c, world, id, rank));
  comm_ = c;
}

RcclComm::~RcclComm() {
  if (comm_) (void)ncclCommDestroy(static_cast<ncclComm_t>(comm_));
}

void RcclComm::allreduce_sum(float *buf, size_t n, hipStream_t s) {
  if (world_ == 1 || n == 0) return;
  count(n * sizeof(float), 2.0);
  PGCN_NCCL(ncclAllReduce(buf, buf, n, ncclFloat32, ncclSum, static_cast<ncclComm_t>(comm_), s));
}

void RcclComm::reduce_scatter_sum(const float *send, float *recv, size_t recvcount,
                                  hipStream_t s) {
  count(recvcount * world_ * sizeof(float), 1.0);
  PGCN_NCCL(ncclReduceScatter(send, recv, recvcount, ncclFloat32, ncclSum,
                              static_cast<ncclComm_t>(comm_), s));
}

void SoloComm::allreduce_sum(float *buf, size_t n, hipStream_t s) {
  (void)buf;
  (void)s;
  if (world_ > 1 && n > 0) count(n * sizeof(float), 2.0);
}

void SoloComm::reduce_scatter_sum(const float *send, float *recv, size_t recvcount,
                                  hipStream_t s) {
  count(recvcount * world_ * sizeof(float), 1.0);
  PGCN_HIP(hipMemcpyAsync(recv, send + (size_t)rank_ * recvcount, recvcount * sizeof(float),
                          hipMemcpyDeviceToDevice, s));
}

// ------------------------------------------------------------------------------------------
// Loopback (in-process) collectives
// ------------------------------------------------------------------------------------------
struct LoopbackGroup::Impl {
  std::mutex mu;
  std::condition_variable cv;
  long long generation = 0;  // completed rendezvous
  int arrived = 0;
  std::vector<const void *> ptrs;
  std::vector<hipEvent_t> evs;
  std::vector<const void *> out_ptrs;  // the last completed rendezvous
  std::vector<hipEvent_t> out_evs;
};

LoopbackGroup::LoopbackGroup(int world) : impl_(std::make_shared<Impl>()), world_(world) {
  PGCN_CHECK(world >= 1 && world <= kLoopbackMaxRanks, PGCN_E_INVALID,
             "loopback group: world must be in [1, 16]");
  impl_->ptrs.assign((size_t)world, nullptr);
  impl_->evs.assign((size_t)world, nullptr);
}

void LoopbackGroup::exchange(int rank, const void *ptr, hipEvent_t ev,
                             std::vector<const void *> *ptrs, std::vector<hipEvent_t> *evs) {
  Impl &m = *impl_;
  std::unique_lock<std::mutex> lk(m.mu);
  const long long gen = m.generation;
  m.ptrs[(size_t)rank] = ptr;
  m.evs[(size_t)rank] = ev;
  if (++m.arrived == world_) {
    m.out_ptrs = m.ptrs;
    m.out_evs = m.evs;
    m.arrived = 0;
    m.generation++;
    m.cv.notify_all();
  } else {
    const bool ok = m.cv.wait_for(lk, std::chrono::duration<double>(timeout_s),
                                  [&] { return m.generation != gen; });
    if (!ok) {
      m.arrived--;
      throw Error(PGCN_E_COMM, "loopback collective: peers did not arrive (rank " +
                                   std::to_string(rank) + ")");
    }
  }
  // the next rendezvous cannot complete before this rank arrives again, so out_* is stable
  *ptrs = m.out_ptrs;
  *evs = m.out_evs;
}

LoopbackComm::LoopbackComm(int rank, std::shared_ptr<LoopbackGroup> group)
    : Comm(rank, group->world()), group_(std::move(group)) {
  PGCN_CHECK(rank >= 0 && rank < world_, PGCN_E_INVALID, "loopback comm: rank");
  PGCN_HIP(hipEventCreateWithFlags(&ready_, hipEventDisableTiming));
  PGCN_HIP(hipEventCreateWithFlags(&done_, hipEventDisableTiming));
}

LoopbackComm::~LoopbackComm() {
  if (ready_) (void)hipEventDestroy(ready_);
  if (done_) (void)hipEventDestroy(done_);
  if (tmp_) (void)hipFree(tmp_);
}

// dst[0, count) = sum over ranks q (in rank order) of send_q[src_offset, src_offset + count)
void LoopbackComm::collective(const float *send, float *dst, size_t count, size_t src_offset,
                              hipStream_t s) {
  std::vector<const void *> ptrs;
  std::vector<hipEvent_t> evs;
  PGCN_HIP(hipEventRecord(ready_, s));  // this rank's send buffer is complete
  group_->exchange(rank_, send, ready_, &ptrs, &evs);
  LoopbackSrcs srcs{};
  for (int q = 0; q < world_; q++) {
    if (q != rank_) PGCN_HIP(hipStreamWaitEvent(s, evs[(size_t)q], 0));
    srcs.p[q] = static_cast<const float *>(ptrs[(size_t)q]) + src_offset;
  }
  srcs.n = world_;
  launch_loopback_sum(srcs, dst, count, s);
  PGCN_HIP(hipEventRecord(done_, s));  // this rank has read every peer's buffer
  group_->exchange(rank_, nullptr, done_, &ptrs, &evs);
  for (int q = 0; q < world_; q++)
    if (q != rank_) PGCN_HIP(hipStreamWaitEvent(s, evs[(size_t)q], 0));
}

void LoopbackComm::allreduce_sum(float *buf, size_t n, hipStream_t s) {
  if (world_ == 1 || n == 0) return;
  count(n * sizeof(float), 2.0);
  if (tmp_n_ < n) {
    if (tmp_) PGCN_HIP(hipFree(tmp_));
    tmp_ = nullptr;
    PGCN_HIP(hipMalloc(&tmp_, n * sizeof(float)));
    tmp_n_ = n;
  }
  // every peer has read `buf` once collective() returns on the stream: then overwrite it
  collective(buf, tmp_, n, 0, s);
  PGCN_HIP(hipMemcpyAsync(buf, tmp_, n * sizeof(float), hipMemcpyDeviceToDevice, s));
}

void LoopbackComm::reduce_scatter_sum(const float *send, float *recv, size_t recvcount,
                                      hipStream_t s) {
  count(recvcount * world_ * sizeof(float), 1.0);
  collective(send, recv, recvcount, (size_t)rank_ * recvcount, s);
}

}  // namespace pgcn
