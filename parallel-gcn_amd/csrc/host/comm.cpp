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

int g_peer_uncached = 0;

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
  enter(s);
  if (world_ == 1 || n == 0) return;
  count(n * sizeof(float), 2.0);
  PGCN_NCCL(ncclAllReduce(buf, buf, n, ncclFloat32, ncclSum, static_cast<ncclComm_t>(comm_), s));
}

void RcclComm::reduce_scatter_sum(const float *send, float *recv, size_t recvcount,
                                  hipStream_t s) {
  enter(s);
  count(recvcount * world_ * sizeof(float), 1.0);
  PGCN_NCCL(ncclReduceScatter(send, recv, recvcount, ncclFloat32, ncclSum,
                              static_cast<ncclComm_t>(comm_), s));
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
  PGCN_CHECK(world >= 1 && world <= kPeerMaxRanks, PGCN_E_INVALID,
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

}  // namespace pgcn

namespace pgcn {

// ------------------------------------------------------------------------------------------
// Peer-mapped collectives (k_peer.hip)
// ------------------------------------------------------------------------------------------
void LoopbackGroup::barrier(int rank) {
  std::vector<const void *> ptrs;
  std::vector<hipEvent_t> evs;
  exchange(rank, nullptr, nullptr, &ptrs, &evs);
}

void LoopbackGroup::allgather(int rank, const void *mine, size_t bytes, void *all) {
  std::vector<const void *> ptrs;
  std::vector<hipEvent_t> evs;
  exchange(rank, mine, nullptr, &ptrs, &evs);
  for (int q = 0; q < world_; q++)
    std::memcpy(static_cast<char *>(all) + (size_t)q * bytes, ptrs[(size_t)q], bytes);
  exchange(rank, nullptr, nullptr, &ptrs, &evs);  // every rank has copied: `mine` may go
}

namespace {
// header (uncached): [flags: kPeerMaxRanks words][arrival counter][error word], 4 KB
constexpr size_t kPeerHeader = 4096;
constexpr size_t kArriveOff = kPeerMaxRanks * 4, kErrOff = kArriveOff + 4;

struct PeerBlob {  // what a rank publishes at construction
  hipIpcMemHandle_t slots, header;
  unsigned long long slots_ptr, header_ptr;  // in-process: the regions' device addresses
  int ok;
  int pad;
};
}  // namespace

PeerComm::PeerComm(int rank, int world, size_t slot_floats, AllGather ag, bool ipc,
                   std::function<void()> host_order, bool solo)
    : Comm(rank, world), ag_(std::move(ag)), ipc_(ipc && !solo), solo_(solo),
      host_order_(std::move(host_order)) {
  PGCN_CHECK(world >= 1 && world <= kPeerMaxRanks && rank >= 0 && rank < world && (ag_ || solo),
             PGCN_E_INVALID, "peer comm: rank / world");
  slot_floats_ = (std::max<size_t>(slot_floats, 4) + 63) / 64 * 64;  // 256-B aligned slots
  bytes_ = 2 * (size_t)world * slot_floats_ * sizeof(float);
  // slots: plain device memory (pushed with plain stores and one system-scope release per
  // pushing workgroup; read after a system-scope acquire: peer_sync.hpp), or uncached
  // (peer_uncached); header: uncached (the flags and counters every rank polls and adds to)
  void *p = nullptr;
  uncached_ = g_peer_uncached != 0 && !solo;
  if (uncached_)
    PGCN_HIP(hipExtMallocWithFlags(&p, bytes_, hipDeviceMallocUncached));
  else
    PGCN_HIP(hipMalloc(&p, bytes_));
  slots_ = static_cast<char *>(p);
  p = nullptr;
  if (hipExtMallocWithFlags(&p, kPeerHeader, hipDeviceMallocUncached) != hipSuccess || !p) {
    (void)hipFree(slots_);
    throw Error(PGCN_E_NOMEM, "peer comm: uncached flag region");
  }
  header_ = static_cast<char *>(p);
  PGCN_HIP(hipMemset(header_, 0, kPeerHeader));
  PGCN_HIP(hipDeviceSynchronize());
  if (solo_) {
    peer_slots_.assign((size_t)world, slots_);
    peer_header_.assign((size_t)world, header_);
    return;
  }
  PeerBlob mine{};
  mine.slots_ptr = (unsigned long long)(uintptr_t)slots_;
  mine.header_ptr = (unsigned long long)(uintptr_t)header_;
  mine.ok = 1;
  if (ipc_ && (hipIpcGetMemHandle(&mine.slots, slots_) != hipSuccess ||
               hipIpcGetMemHandle(&mine.header, header_) != hipSuccess))
    mine.ok = 0;
  std::vector<PeerBlob> all((size_t)world);
  ag_(&mine, sizeof mine, all.data());
  // every rank reports whether it could map every peer; all fail together
  int ok = 1;
  std::string why;
  for (int q = 0; q < world; q++) ok &= all[(size_t)q].ok;
  if (!ok) why = "a rank could not export its regions";
  peer_slots_.assign((size_t)world, nullptr);
  peer_header_.assign((size_t)world, nullptr);
  for (int q = 0; q < world && ok; q++) {
    if (q == rank || !ipc_) {
      peer_slots_[(size_t)q] = q == rank ? slots_ : reinterpret_cast<char *>((uintptr_t)all[(size_t)q].slots_ptr);
      peer_header_[(size_t)q] = q == rank ? header_ : reinterpret_cast<char *>((uintptr_t)all[(size_t)q].header_ptr);
      continue;
    }
    for (int h = 0; h < 2 && ok; h++) {
      void *m = nullptr;
      const hipError_t e = hipIpcOpenMemHandle(&m, h ? all[(size_t)q].header : all[(size_t)q].slots,
                                               hipIpcMemLazyEnablePeerAccess);
      if (e != hipSuccess || !m) {
        ok = 0;
        why = std::string("hipIpcOpenMemHandle of rank ") + std::to_string(q) + ": " + hipGetErrorString(e);
        break;
      }
      (h ? peer_header_ : peer_slots_)[(size_t)q] = static_cast<char *>(m);
    }
  }
  int oks[kPeerMaxRanks];
  ag_(&ok, sizeof ok, oks);
  for (int q = 0; q < world; q++) ok &= oks[q];
  if (!ok) {
    unmap();
    (void)hipFree(slots_);
    (void)hipFree(header_);
    slots_ = header_ = nullptr;
    throw Error(PGCN_E_COMM, "peer comm: " + (why.empty() ? std::string("a peer failed to map") : why));
  }
}

void PeerComm::host_barrier() {
  if (solo_ || !ag_) return;
  int token = 0;
  std::vector<int> all((size_t)world_);
  ag_(&token, sizeof token, all.data());
}

void PeerComm::unmap() {
  if (ipc_)
    for (int q = 0; q < world_; q++) {
      if (q == rank_) continue;
      if (q < (int)peer_slots_.size() && peer_slots_[(size_t)q]) (void)hipIpcCloseMemHandle(peer_slots_[(size_t)q]);
      if (q < (int)peer_header_.size() && peer_header_[(size_t)q]) (void)hipIpcCloseMemHandle(peer_header_[(size_t)q]);
    }
  peer_slots_.clear();
  peer_header_.clear();
}

PeerComm::~PeerComm() {
  if (!slots_) return;
  (void)hipDeviceSynchronize();
  if (!solo_) {
    // nobody closes or frees before every rank is done with every collective, and nobody
    // frees before every peer has closed its mappings of this rank's regions
    int token = 0;
    std::vector<int> all((size_t)world_);
    try {
      ag_(&token, sizeof token, all.data());
    } catch (...) {
    }
    unmap();
    try {
      ag_(&token, sizeof token, all.data());
    } catch (...) {
    }
  }
  (void)hipFree(slots_);
  (void)hipFree(header_);
}

float *PeerComm::slot(char *slots, int parity, int sender) const {
  return reinterpret_cast<float *>(slots) + ((size_t)parity * world_ + (size_t)sender) * slot_floats_;
}

PeerSink PeerComm::sink(int rows_per_rank, size_t row_floats) {
  PGCN_CHECK((size_t)rows_per_rank * row_floats <= slot_floats_, PGCN_E_INVALID,
             "peer comm: collective larger than its slots");
  const unsigned g = ++gen_;
  PeerSink k{};
  for (int q = 0; q < world_; q++) {
    k.dst[q] = slot(peer_slots_[(size_t)q], (int)(g & 1), rank_);
    k.flag[q] = reinterpret_cast<unsigned *>(peer_header_[(size_t)q]) + rank_;
  }
  k.arrive = reinterpret_cast<unsigned *>(header_ + kArriveOff);
  k.slot_bytes = (long long)(slot_floats_ * sizeof(float));
  k.gen = g;
  k.world = world_;
  k.rows_per_rank = rows_per_rank;
  k.signal = 1;
  if (!host_order_) {
    // separate processes (or solo): the push launch's last workgroup waits (wait() adds none:
    // W = 8 / 4 solo rank epochs 0.483 / 0.667 ms against 0.486 / 0.674 with the one-wave wait
    // kernel, three interleaved pairs, profiles/r05/u);
    // in-process ranks may share a hardware queue, where that spin could block a peer's push
    k.wait_flags = reinterpret_cast<const unsigned *>(header_) + (solo_ ? rank_ : 0);
    k.nwait = solo_ ? 1 : world_;
    k.err = reinterpret_cast<unsigned *>(header_ + kErrOff);
  }
  return k;
}

void PeerComm::wait(hipStream_t s) {
  if (!host_order_) return;  // fused into the push (sink)
  host_order_();
  // (solo: every push signalled this rank's own flag word only)
  launch_peer_wait(reinterpret_cast<const unsigned *>(header_) + (solo_ ? rank_ : 0),
                   solo_ ? 1 : world_, gen_, reinterpret_cast<unsigned *>(header_ + kErrOff), s);
}

PeerRecv PeerComm::recv() const {
  PeerRecv r{};
  for (int q = 0; q < world_; q++) r.slot[q] = slot(slots_, (int)(gen_ & 1), q);
  r.world = world_;
  return r;
}

void PeerComm::check() const {
  unsigned e = 0;
  PGCN_HIP(hipMemcpy(&e, header_ + kErrOff, sizeof e, hipMemcpyDeviceToHost));
  if (e)
    throw Error(PGCN_E_COMM, "peer exchange: rank " + std::to_string(e & 0xffff) +
                                 " did not signal rank " + std::to_string(rank_) + " in time");
}

bool PeerComm::small_allreduce(size_t n, PeerSmall *p) {
  if (world_ == 1 || n == 0 || host_order_ || n > (size_t)kPeerSmallAllreduce) return false;
  count(n * sizeof(float), 2.0);
  p->k = sink(1, n);
  p->r = recv();
  p->waited = reinterpret_cast<const unsigned *>(header_) + (solo_ ? rank_ : 0);
  p->nwait = solo_ ? 1 : world_;
  p->err = reinterpret_cast<unsigned *>(header_ + kErrOff);
  return true;
}

void PeerComm::allreduce_sum(float *buf, size_t n, hipStream_t s) {
  enter(s);
  PeerSmall p;
  if (small_allreduce(n, &p)) {
    // separate processes (or solo): push, wait and sum in one workgroup
    launch_peer_allreduce_small(buf, (int)n, p.k, p.r, p.waited, p.nwait, p.err, s);
    return;
  }
  if (world_ == 1 || n == 0) return;
  count(n * sizeof(float), 2.0);
  PeerSink k = sink(1, n);
  // every receiver gets the same n floats: send[q * n ..) = buf for every q (stride 0)
  k.rows_per_rank = 0;
  launch_peer_push(buf, n, k, s, /*same_for_all=*/true);
  wait(s);
  launch_peer_sum(recv(), buf, n, s);
}

bool PeerComm::allreduce_grads(float *buf, size_t n, const GradRegions &r, hipStream_t s,
                               PeerRecv *rv) {
  if (host_order_ || world_ == 1 || n == 0) return false;
  enter(s);
  count(n * sizeof(float), 2.0);
  PeerSink k = sink(1, n);
  k.rows_per_rank = 0;  // every receiver gets the same n floats
  launch_peer_push_grads(buf, (long long)n, r, k, s);
  *rv = recv();
  return true;
}

void PeerComm::reduce_scatter_sum(const float *send, float *recv_buf, size_t recvcount,
                                  hipStream_t s) {
  enter(s);
  count(recvcount * world_ * sizeof(float), 1.0);
  PeerSink k = sink(1, recvcount);
  launch_peer_push(send, recvcount, k, s, false);
  wait(s);
  launch_peer_sum(recv(), recv_buf, recvcount, s);
}

}  // namespace pgcn
