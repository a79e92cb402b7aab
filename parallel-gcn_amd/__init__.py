"""parallel-gcn_amd -- Python host glue for the MI355X GCN engine (libpgcn.so).

The product is C++/HIP: kernels + host classes behind the C ABI in include/pgcn.h.  This
module only binds that ABI with ctypes so tests, bench.py and __graft_entry__ can drive it;
it mirrors the reference's host interface for the path (src/main.cpp:9-61,
include/gcn.cuh:79-122): load a dataset with the kept hpdga Parser, build a GCN, call
train_epoch() / eval(split) / run().

There is no CPU fallback: importing this module without the built library raises, and
creating an engine without a HIP device raises PgcnError(PGCN_E_NODEVICE).
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# PGCN_LIB: another build of the library (A/B experiments); the default is the in-tree build
LIB_PATH = os.environ.get("PGCN_LIB") or os.path.join(HERE, "libpgcn.so")

PGCN_OK = 0
PGCN_E_INVALID = -1
PGCN_E_NOMEM = -2
PGCN_E_IO = -3
PGCN_E_COMM = -4
PGCN_E_NODEVICE = -5
MAX_LAYERS = 16

if not os.path.exists(LIB_PATH):
    raise ImportError(f"{LIB_PATH} is not built: run `make -C parallel-gcn_amd` "
                      "(or __graft_entry__.build()); there is no fallback path")
lib = ctypes.CDLL(LIB_PATH)

c_int, c_ll, c_float, c_void_p = ctypes.c_int, ctypes.c_longlong, ctypes.c_float, ctypes.c_void_p
c_size_t, c_u64, c_double = ctypes.c_size_t, ctypes.c_uint64, ctypes.c_double
P = ctypes.POINTER


class PgcnParams(ctypes.Structure):
    _fields_ = [("num_nodes", c_int), ("input_dim", c_int), ("output_dim", c_int),
                ("n_layers", c_int), ("hidden_dims", c_int * MAX_LAYERS),
                ("dropouts", c_float * MAX_LAYERS), ("epochs", c_int), ("early_stopping", c_int),
                ("learning_rate", c_float), ("weight_decay", c_float), ("beta1", c_float),
                ("beta2", c_float), ("eps", c_float), ("reassociate_last", c_int),
                ("seed", ctypes.c_uint)]


class PgcnData(ctypes.Structure):
    _fields_ = [("num_nodes", c_int), ("graph_indptr", P(c_int)), ("graph_indices", P(c_int)),
                ("feat_indptr", P(c_int)), ("feat_indices", P(c_int)),
                ("feat_values", P(c_float)), ("label", P(c_int)), ("split", P(c_int))]


def _sig(name, res, *args):
    if os.environ.get("PGCN_LIB") and not hasattr(lib, name):
        return None  # an A/B build from before this entry point: the bench does not call it
    f = getattr(lib, name)
    f.restype = res
    f.argtypes = list(args)
    return f


_sig("pgcn_status_string", ctypes.c_char_p, c_int)
_sig("pgcn_version", c_int)
_sig("pgcn_rng_seed", None, P(c_u64))
_sig("pgcn_rng_seed_glibc", None, ctypes.c_uint, P(c_u64))
_sig("pgcn_rng_jump", None, P(c_u64), c_u64)
_sig("pgcn_rng_jump_table", c_int, c_u64, c_void_p)
_sig("pgcn_graph_create", c_int, c_int, c_void_p, c_void_p, P(c_void_p))
_sig("pgcn_graph_create_values", c_int, c_int, c_void_p, c_void_p, c_void_p, P(c_void_p))
_sig("pgcn_graph_destroy", c_int, c_void_p)
_sig("pgcn_graph_nnz", c_ll, c_void_p)
_sig("pgcn_graphsum", c_int, c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_void_p)
_sig("pgcn_gemm", c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_int, c_int, c_void_p,
     c_int, c_void_p, c_ll, c_ll, c_float, c_void_p)
_sig("pgcn_gemm_tn_workspace", c_size_t, c_int, c_int, c_int)
_sig("pgcn_gemm_tn", c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_int, c_void_p,
     c_int, c_void_p, c_ll, c_ll, c_float, c_void_p, c_void_p)
_sig("pgcn_mask_nibbles", c_int, c_void_p, c_ll, c_ll, c_int, c_int, c_void_p, c_void_p)
_sig("pgcn_gemm_xstream", c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_int, c_int,
     c_void_p, c_int, c_void_p, c_float, c_void_p)
_sig("pgcn_gemm_xstream_dual", c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_int,
     c_int, c_void_p, c_void_p, c_int, c_void_p, c_float, c_void_p)
_sig("pgcn_gemm_tn_xstream", c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_int,
     c_void_p, c_int, c_void_p, c_float, c_void_p, c_void_p)
_sig("pgcn_gemm_xstream_flat", c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_int,
     c_int, c_void_p, c_void_p, c_int, c_void_p, c_ll, c_ll, c_float, c_void_p)
_sig("pgcn_gemm_tn_xstream_flat", c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_int,
     c_void_p, c_int, c_void_p, c_ll, c_ll, c_float, c_void_p, c_void_p)
_sig("pgcn_spmm_csr", c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_float,
     c_void_p, c_void_p, c_void_p)
_sig("pgcn_spmm_csc_bwd", c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
     c_float, c_void_p, c_void_p, c_void_p)
_sig("pgcn_csr_transpose", c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p)
_sig("pgcn_dropout_mask", c_int, c_void_p, c_ll, c_ll, c_ll, c_float, c_void_p, c_void_p, c_void_p)
_sig("pgcn_dropout_apply", c_int, c_void_p, c_ll, c_void_p, c_float, c_void_p)
_sig("pgcn_relu_fwd", c_int, c_void_p, c_ll, c_void_p, c_int, c_void_p)
_sig("pgcn_relu_bwd", c_int, c_void_p, c_ll, c_void_p, c_void_p)
_sig("pgcn_xent_blocks", c_int, c_int)
_sig("pgcn_xent_fwd", c_int, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
     c_void_p, c_void_p)
_sig("pgcn_finalize", c_int, c_void_p, c_int, c_int, c_void_p, c_ll, c_float, c_void_p, c_void_p)
_sig("pgcn_adam", c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_ll, c_float, c_float, c_float,
     c_float, c_float, c_int, c_void_p)
_sig("pgcn_adam_step_size", c_float, c_float, c_float, c_float, c_int)
_sig("pgcn_params_default", None, P(PgcnParams))
_sig("pgcn_gcn_create", c_int, P(PgcnParams), P(PgcnData), c_int, P(c_void_p))
_sig("pgcn_comm_unique_id", c_int, c_void_p)
_sig("pgcn_gcn_create_dist", c_int, P(PgcnParams), P(PgcnData), c_int, c_int, c_int, c_void_p,
     P(c_void_p))
_sig("pgcn_gcn_destroy", c_int, c_void_p)
# the caller's host all-gather for the peer-mapped engine (pgcn_allgather_fn)
ALLGATHER_FN = ctypes.CFUNCTYPE(c_int, c_void_p, ctypes.c_size_t, c_void_p, c_void_p)
_sig("pgcn_gcn_create_peer", c_int, P(PgcnParams), P(PgcnData), c_int, c_int, c_int,
     ALLGATHER_FN, c_void_p, P(c_void_p))
_sig("pgcn_loopback_create", c_int, c_int, P(c_void_p))
_sig("pgcn_debug_gcn_create_solo", c_int, P(PgcnParams), P(PgcnData), c_int, c_int, c_int,
     P(c_void_p))
_sig("pgcn_loopback_destroy", c_int, c_void_p)
_sig("pgcn_gcn_create_loopback", c_int, P(PgcnParams), P(PgcnData), c_int, c_int, c_void_p,
     P(c_void_p))
_sig("pgcn_gcn_query", c_ll, c_void_p, ctypes.c_char_p)
_sig("pgcn_gcn_train_epoch", c_int, c_void_p, P(c_float))
_sig("pgcn_gcn_eval", c_int, c_void_p, c_int, P(c_float))
_sig("pgcn_gcn_epoch_async", c_int, c_void_p)
_sig("pgcn_gcn_sync", c_int, c_void_p)
_sig("pgcn_gcn_results", c_int, c_void_p, c_int, P(c_float))
_sig("pgcn_gcn_run", c_int, c_void_p, c_int)
_sig("pgcn_gcn_get_var", c_ll, c_void_p, c_int, c_int, P(c_float))
_sig("pgcn_gcn_num_vars", c_int, c_void_p)
_sig("pgcn_gcn_profile", c_int, c_void_p, c_int)
_sig("pgcn_gcn_profile_read", c_int, c_void_p, P(c_double), P(c_ll), P(c_double))
_sig("pgcn_gcn_profile_read_mm", c_int, c_void_p, P(c_double), P(c_ll), P(c_double))
_sig("pgcn_gcn_node_range", c_int, c_void_p, P(c_int), P(c_int))
_sig("pgcn_dataset_load", c_int, ctypes.c_char_p, ctypes.c_char_p, P(c_void_p))
_sig("pgcn_dataset_load_cached", c_int, ctypes.c_char_p, ctypes.c_char_p, P(c_void_p), P(c_int))
_sig("pgcn_dataset_save", c_int, c_void_p, ctypes.c_char_p)
_sig("pgcn_dataset_binarize", c_int, c_void_p)
_sig("pgcn_dataset_load_binary", c_int, ctypes.c_char_p, P(c_void_p))
_sig("pgcn_dataset_synthetic", c_int, c_int, c_int, c_int, c_ll, c_u64, P(c_void_p))
_sig("pgcn_dataset_view", c_int, c_void_p, P(PgcnData), P(c_int), P(c_int))
_sig("pgcn_dataset_free", c_int, c_void_p)
_sig("pgcn_debug_set", c_int, ctypes.c_char_p, c_int)
_sig("pgcn_debug_path_count", c_ll, ctypes.c_char_p, c_int)
_sig("pgcn_debug_empty_launches", c_int, c_int, c_void_p)
_sig("pgcn_debug_exp_check", c_int, c_void_p, c_ll, c_void_p, c_void_p, c_void_p)
_sig("pgcn_debug_div_check", c_int, c_void_p, c_void_p, c_ll, c_void_p, c_void_p)
_sig("pgcn_debug_lds_check", c_int, c_int, c_int, c_void_p, c_void_p, c_int, P(ctypes.c_double),
     P(c_ll))
_sig("pgcn_debug_lds_counts", c_ll, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p, c_ll,
     c_void_p)
_sig("pgcn_partition_bounds", c_int, c_int, c_void_p, c_int, c_void_p, P(c_int))
_sig("pgcn_debug_rank_graph", c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
     c_void_p, c_void_p, c_void_p)
_sig("pgcn_partition_subgraph", c_ll, c_int, c_void_p, c_void_p, c_int, c_int, c_void_p,
     c_void_p, c_void_p)


class PgcnError(RuntimeError):
    def __init__(self, status, where=""):
        self.status = status
        super().__init__(f"{where}: {lib.pgcn_status_string(status).decode()} ({status})")


def check(status, where=""):
    if status != PGCN_OK:
        raise PgcnError(status, where)
    return status


def _ptr(a):
    return a.ctypes.data_as(c_void_p)


KERNEL_PATHS = ("xs_nn_ring", "xs_tn_ring", "xs_nn", "xs_tn", "gs_ring", "gs_gather", "out_xent",
                "gemm_nn", "gemm_tn", "gemm_nn_w", "gemm_tn_w", "launches")


def path_counts(reset=False, thread=False):
    """Launch counts of the kernel families since the last reset (pgcn_debug_path_count);
    thread: the calling host thread's launches only (a loopback rank's own)."""
    out = {}
    t = 2 if thread else 0
    for k in KERNEL_PATHS:
        n = lib.pgcn_debug_path_count(k.encode(), t)
        if n < 0:
            raise PgcnError(int(n), "path_count " + k)
        out[k] = int(n)
    if reset:
        lib.pgcn_debug_path_count(None, 1 | t)
    return out


def reset_path_counts(thread=False):
    check(int(lib.pgcn_debug_path_count(None, 3 if thread else 1)), "path_count reset")


# --------------------------------------------------------------------------- data
class Dataset:
    """GCNData (include/gcn.cuh:51-58) owned by libpgcn: the hpdga loader or the synthetic
    reddit-shaped generator.  Arrays are exposed as zero-copy numpy views."""

    def __init__(self, handle):
        self._h = c_void_p(handle)
        self.view = PgcnData()
        fi, fo = c_int(), c_int()
        check(lib.pgcn_dataset_view(self._h, ctypes.byref(self.view), ctypes.byref(fi),
                                    ctypes.byref(fo)), "dataset_view")
        self.input_dim, self.output_dim = fi.value, fo.value
        self.num_nodes = self.view.num_nodes
        n = self.num_nodes

        def arr(p, count, dt):
            if count == 0:
                return np.zeros(0, dt)
            return np.ctypeslib.as_array(ctypes.cast(p, P(ctypes.c_int if dt == np.int32 else c_float)),
                                         shape=(count,))
        self.graph_indptr = arr(self.view.graph_indptr, n + 1, np.int32)
        self.graph_indices = arr(self.view.graph_indices, int(self.graph_indptr[-1]), np.int32)
        self.feat_indptr = arr(self.view.feat_indptr, n + 1, np.int32)
        nnzx = int(self.feat_indptr[-1])
        self.feat_indices = arr(self.view.feat_indices, nnzx, np.int32)
        self.feat_values = arr(self.view.feat_values, nnzx, np.float32)
        self.label = arr(self.view.label, n, np.int32)
        self.split = arr(self.view.split, n, np.int32)

    @staticmethod
    def load(root, name):
        """Parser(&params, &data, name).parse() with data/<name>.* under root."""
        h = c_void_p()
        check(lib.pgcn_dataset_load(root.encode(), name.encode(), ctypes.byref(h)),
              f"Cannot read input: {name}")
        return Dataset(h.value)

    @staticmethod
    def load_cached(root, name):
        """load() through the binary cache data/<name>.pgcnbin (written on a miss).
        Returns (dataset, from_cache)."""
        h, hit = c_void_p(), c_int()
        check(lib.pgcn_dataset_load_cached(root.encode(), name.encode(), ctypes.byref(h),
                                           ctypes.byref(hit)), f"Cannot read input: {name}")
        return Dataset(h.value), bool(hit.value)

    def binarize(self):
        """PART2 NO_FEATURE (src/parser.cpp:100-104): every feature value becomes 1.0 (the
        arrays of this object are views, so they change in place)."""
        check(lib.pgcn_dataset_binarize(self._h), "dataset_binarize")

    def save(self, path):
        check(lib.pgcn_dataset_save(self._h, path.encode()), f"dataset_save {path}")

    @staticmethod
    def load_binary(path):
        h = c_void_p()
        check(lib.pgcn_dataset_load_binary(path.encode(), ctypes.byref(h)),
              f"dataset_load_binary {path}")
        return Dataset(h.value)

    @staticmethod
    def synthetic(n, f, c, undirected_edges, seed=1):
        h = c_void_p()
        check(lib.pgcn_dataset_synthetic(n, f, c, undirected_edges, seed, ctypes.byref(h)),
              "dataset_synthetic")
        return Dataset(h.value)

    def __del__(self):
        # (at interpreter exit the module's globals may already be gone: nothing to free then)
        if getattr(self, "_h", None) and self._h.value and lib is not None:
            lib.pgcn_dataset_free(self._h)
            self._h = c_void_p()


def make_params(ds, hidden_dims=(16,), dropouts=(0.5, 0.5), epochs=100, early_stopping=0,
                learning_rate=0.01, weight_decay=5e-4, beta1=0.9, beta2=0.999, eps=1e-8,
                reassociate_last=True, seed=0):
    p = PgcnParams()
    lib.pgcn_params_default(ctypes.byref(p))
    p.reassociate_last = 1 if reassociate_last else 0
    p.seed = seed
    p.num_nodes, p.input_dim, p.output_dim = ds.num_nodes, ds.input_dim, ds.output_dim
    p.n_layers = len(hidden_dims) + 1
    assert len(dropouts) == p.n_layers
    for i, h in enumerate(hidden_dims):
        p.hidden_dims[i] = h
    for i, d in enumerate(dropouts):
        p.dropouts[i] = d
    p.epochs, p.early_stopping = epochs, early_stopping
    p.learning_rate, p.weight_decay, p.beta1, p.beta2, p.eps = (learning_rate, weight_decay,
                                                               beta1, beta2, eps)
    return p


# --------------------------------------------------------------------------- engine
class GCN:
    """GCN(params, data) of include/gcn.cuh:79-122 on one GPU, or the edge-cut variant when
    rank/world/unique_id are given (one process per GPU)."""

    def __init__(self, params, ds, device=0, rank=None, world=None, unique_id=None,
                 loopback=None, solo=False, allgather=None):
        self.ds = ds  # keep the host data alive while the engine is built
        h = c_void_p()
        self._ag = None
        if allgather is not None:
            # peer-mapped exchange (pgcn_gcn_create_peer): allgather(bytes) -> [bytes of every
            # rank], called at creation and at close (kept alive with the engine)
            self._ag = peer_allgather_fn(allgather)
            check(lib.pgcn_gcn_create_peer(ctypes.byref(params), ctypes.byref(ds.view), device,
                                           rank, world, self._ag, None, ctypes.byref(h)),
                  "gcn_create_peer")
        elif solo:  # timing only: rank `rank` of `world` with no peers (pgcn_debug_gcn_create_solo)
            check(lib.pgcn_debug_gcn_create_solo(ctypes.byref(params), ctypes.byref(ds.view),
                                                 device, rank, world, ctypes.byref(h)),
                  "gcn_create_solo")
        elif loopback is not None:
            check(lib.pgcn_gcn_create_loopback(ctypes.byref(params), ctypes.byref(ds.view),
                                               device, rank, loopback._h, ctypes.byref(h)),
                  "gcn_create_loopback")
        elif world is None:
            check(lib.pgcn_gcn_create(ctypes.byref(params), ctypes.byref(ds.view), device,
                                      ctypes.byref(h)), "gcn_create")
        else:
            uid = ctypes.create_string_buffer(bytes(unique_id), 128)
            check(lib.pgcn_gcn_create_dist(ctypes.byref(params), ctypes.byref(ds.view), device,
                                           rank, world, uid, ctypes.byref(h)), "gcn_create_dist")
        self._h = h
        self.params = params

    def train_epoch(self):
        out = (c_float * 2)()
        check(lib.pgcn_gcn_train_epoch(self._h, out), "train_epoch")
        return out[0], out[1]

    def eval(self, split):
        out = (c_float * 2)()
        check(lib.pgcn_gcn_eval(self._h, split, out), "eval")
        return out[0], out[1]

    def epoch_async(self):
        check(lib.pgcn_gcn_epoch_async(self._h), "epoch_async")

    def sync(self):
        check(lib.pgcn_gcn_sync(self._h), "sync")

    def results(self, n):
        """The last min(n, epochs run, 1024) epoch lines [train_loss, train_acc, val_loss,
        val_acc], oldest first."""
        out = np.zeros(4 * max(n, 0), np.float32)
        rows = lib.pgcn_gcn_results(self._h, n, out.ctypes.data_as(P(c_float)))
        if rows < 0:
            raise PgcnError(rows, "results")
        return out[:4 * rows].reshape(rows, 4)

    def run(self, verbose=True):
        check(lib.pgcn_gcn_run(self._h, 1 if verbose else 0), "run")

    def num_vars(self):
        return lib.pgcn_gcn_num_vars(self._h)

    def get_var(self, idx, which=0):
        n = lib.pgcn_gcn_get_var(self._h, idx, which, None)
        if n < 0:
            raise PgcnError(int(n), "get_var")
        out = np.zeros(n, np.float32)
        if n:
            lib.pgcn_gcn_get_var(self._h, idx, which, out.ctypes.data_as(P(c_float)))
        return out

    def profile(self, on):
        check(lib.pgcn_gcn_profile(self._h, 1 if on else 0), "profile")

    def profile_read(self):
        ms, calls, byts = c_double(), c_ll(), c_double()
        check(lib.pgcn_gcn_profile_read(self._h, ctypes.byref(ms), ctypes.byref(calls),
                                        ctypes.byref(byts)), "profile_read")
        return ms.value, calls.value, byts.value

    def profile_read_mm(self):
        """(ms, launches, flops) of the profiled XW contractions (MFMA kernels)."""
        ms, calls, fl = c_double(), c_ll(), c_double()
        check(lib.pgcn_gcn_profile_read_mm(self._h, ctypes.byref(ms), ctypes.byref(calls),
                                           ctypes.byref(fl)), "profile_read_mm")
        return ms.value, calls.value, fl.value

    def query(self, key):
        """Engine facts: world, rank, comm (0 none / 1 RCCL / 2 loopback), reassociated,
        graph_symmetric, graphsum_lds, epochs."""
        v = lib.pgcn_gcn_query(self._h, key.encode())
        if v < 0:
            raise PgcnError(int(v), f"query {key}")
        return int(v)

    def node_range(self):
        a, b = c_int(), c_int()
        lib.pgcn_gcn_node_range(self._h, ctypes.byref(a), ctypes.byref(b))
        return a.value, b.value

    def close(self):
        if self._h and self._h.value:
            lib.pgcn_gcn_destroy(self._h)
            self._h = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class LoopbackGroup:
    """`world` in-process edge-cut ranks on one device (pgcn_loopback_create).  Create the
    engines with GCN(..., rank=r, loopback=group), each from its own thread (see run_ranks)."""

    def __init__(self, world):
        h = c_void_p()
        check(lib.pgcn_loopback_create(world, ctypes.byref(h)), "loopback_create")
        self._h = h
        self.world = world

    def __del__(self):
        if getattr(self, "_h", None) and self._h.value:
            lib.pgcn_loopback_destroy(self._h)
            self._h = c_void_p()


def peer_allgather_fn(allgather):
    """A pgcn_allgather_fn over a Python all-gather: allgather(data: bytes) -> list of every
    rank's bytes in rank order (torch.distributed, a TCP store, ...)."""
    def cb(mine, nbytes, out, user):
        try:
            parts = allgather(ctypes.string_at(mine, nbytes))
            buf = b"".join(parts)
            if len(buf) != nbytes * len(parts):
                return -1
            ctypes.memmove(out, buf, len(buf))
            return 0
        except Exception:  # noqa: BLE001 -- reported to the engine as a failed all-gather
            return -1
    return ALLGATHER_FN(cb)


def torch_allgather(group=None):
    """allgather(bytes) over torch.distributed (gloo: CPU tensors)."""
    import torch
    import torch.distributed as dist

    def ag(data):
        n = dist.get_world_size(group)
        t = torch.frombuffer(bytearray(data), dtype=torch.uint8)
        out = [torch.empty_like(t) for _ in range(n)]
        dist.all_gather(out, t, group=group)
        return [bytes(o.numpy().tobytes()) for o in out]
    return ag


def run_ranks(world, fn):
    """Calls fn(rank) for every rank in its own thread (ctypes releases the GIL during the
    engine's calls, so the ranks' collectives rendezvous); returns the results in rank order
    and re-raises the first exception."""
    import threading
    out, err = [None] * world, [None] * world

    def body(r):
        try:
            out[r] = fn(r)
        except BaseException as e:  # noqa: BLE001 -- re-raised below
            err[r] = e
    ts = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for e in err:
        if e is not None:
            raise e
    return out


def comm_unique_id():
    buf = ctypes.create_string_buffer(128)
    check(lib.pgcn_comm_unique_id(buf), "comm_unique_id")
    return buf.raw


# --------------------------------------------------------------------------- host helpers
def rng_seed(seed=0):
    s = (c_u64 * 2)()
    if seed:
        lib.pgcn_rng_seed_glibc(seed, s)
    else:
        lib.pgcn_rng_seed(s)
    return np.array([s[0], s[1]], np.uint64)


def rng_jump(state, k):
    s = (c_u64 * 2)(int(state[0]), int(state[1]))
    lib.pgcn_rng_jump(s, int(k))
    return np.array([s[0], s[1]], np.uint64)


def rng_jump_table(period):
    t = np.zeros(16 * 256 * 2, np.uint64)
    check(lib.pgcn_rng_jump_table(int(period), _ptr(t)), "rng_jump_table")
    return t


def partition_bounds(indptr, world):
    indptr = np.ascontiguousarray(indptr, np.int32)
    b = np.zeros(world + 1, np.int32)
    mr = c_int()
    check(lib.pgcn_partition_bounds(len(indptr) - 1, _ptr(indptr), world, _ptr(b),
                                    ctypes.byref(mr)), "partition_bounds")
    return b, mr.value


def partition_subgraph(indptr, indices, world, rank):
    indptr = np.ascontiguousarray(indptr, np.int32)
    indices = np.ascontiguousarray(indices, np.int32)
    n = len(indptr) - 1
    _, maxrows = partition_bounds(indptr, world)
    nnz = lib.pgcn_partition_subgraph(n, _ptr(indptr), _ptr(indices), world, rank, None, None, None)
    if nnz < 0:
        raise PgcnError(int(nnz), "partition_subgraph")
    sp = np.zeros(world * maxrows + 1, np.int32)
    si = np.zeros(max(nnz, 1), np.int32)
    sv = np.zeros(max(nnz, 1), np.float32)
    lib.pgcn_partition_subgraph(n, _ptr(indptr), _ptr(indices), world, rank, _ptr(sp), _ptr(si),
                                _ptr(sv))
    return sp, si[:nnz], sv[:nnz]


def csr_transpose(indptr, indices, n_cols):
    indptr = np.ascontiguousarray(indptr, np.int32)
    indices = np.ascontiguousarray(indices, np.int32)
    m, nnz = len(indptr) - 1, int(indptr[-1])
    cp = np.zeros(n_cols + 1, np.int32)
    cr = np.zeros(max(nnz, 1), np.int32)
    cpos = np.zeros(max(nnz, 1), np.int32)
    check(lib.pgcn_csr_transpose(m, n_cols, _ptr(indptr), _ptr(indices), _ptr(cp), _ptr(cr),
                                 _ptr(cpos)), "csr_transpose")
    return cp, cr[:nnz], cpos[:nnz]


EXPORTED = [
    "pgcn_status_string", "pgcn_version", "pgcn_rng_seed", "pgcn_rng_seed_glibc", "pgcn_rng_jump",
    "pgcn_graph_create", "pgcn_graph_create_values", "pgcn_debug_rank_graph",
    "pgcn_graph_destroy", "pgcn_graph_nnz", "pgcn_graphsum", "pgcn_gemm", "pgcn_gemm_tn_workspace",
    "pgcn_gemm_tn", "pgcn_mask_nibbles", "pgcn_gemm_xstream", "pgcn_gemm_xstream_dual",
    "pgcn_gemm_tn_xstream", "pgcn_gemm_xstream_flat", "pgcn_gemm_tn_xstream_flat",
    "pgcn_spmm_csr", "pgcn_spmm_csc_bwd", "pgcn_csr_transpose",
    "pgcn_rng_jump_table", "pgcn_dropout_mask", "pgcn_dropout_apply", "pgcn_relu_fwd",
    "pgcn_relu_bwd", "pgcn_xent_blocks", "pgcn_xent_fwd", "pgcn_finalize", "pgcn_adam",
    "pgcn_adam_step_size", "pgcn_params_default", "pgcn_gcn_create", "pgcn_comm_unique_id",
    "pgcn_gcn_create_dist", "pgcn_gcn_create_peer", "pgcn_loopback_create",
    "pgcn_loopback_destroy",
    "pgcn_debug_gcn_create_solo",
    "pgcn_gcn_create_loopback", "pgcn_gcn_query", "pgcn_gcn_destroy", "pgcn_gcn_train_epoch", "pgcn_gcn_eval",
    "pgcn_gcn_epoch_async", "pgcn_gcn_sync", "pgcn_gcn_results", "pgcn_gcn_run",
    "pgcn_gcn_get_var", "pgcn_gcn_num_vars", "pgcn_gcn_profile", "pgcn_gcn_profile_read",
    "pgcn_gcn_profile_read_mm",
    "pgcn_gcn_node_range", "pgcn_dataset_load", "pgcn_dataset_load_cached", "pgcn_dataset_save",
    "pgcn_dataset_load_binary", "pgcn_dataset_binarize", "pgcn_dataset_synthetic",
    "pgcn_dataset_view",
    "pgcn_dataset_free", "pgcn_partition_bounds", "pgcn_partition_subgraph", "pgcn_debug_set",
    "pgcn_debug_lds_check", "pgcn_debug_lds_counts", "pgcn_debug_path_count",
    "pgcn_debug_empty_launches", "pgcn_debug_exp_check", "pgcn_debug_div_check",
]
