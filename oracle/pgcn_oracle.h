/* oracle/pgcn_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the reference's sequential CPU GCN (hpdga-spring23/src/ sources).
 * It is the parity checker for the HIP engine and is pinned bit-for-bit against the
 * reference itself (oracle/_ref, built from the reference sources by oracle/Makefile) by
 * tests/test_oracle_pinned.py on the committed golden fixtures in tests/golden/.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library. The product (parallel-gcn_amd/libpgcn.so) never links or calls it.
 */
#ifndef PGCN_ORACLE_H
#define PGCN_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OR_RAND_MAX 0x7fffffff /* MY_RAND_MAX, hpdga-spring23/include/rand.h:6 */
#define OR_MAX_LAYERS 16

/* ---- RNG: xorshift128+ (hpdga-spring23/src/rand.cpp:6-28) ---- */
void or_rng_seed(uint64_t s[2]);
void or_rng_seed_glibc(unsigned seed, uint64_t s[2]);
uint32_t or_rng_next(uint64_t s[2]);

/* ---- per-op restatements (each cites the reference lines it follows in the .c) ---- */
void or_glorot(float *w, long n, int in_size, int out_size, uint64_t s[2]);
void or_dropout_fwd(float *x, int *mask, long n, float p, uint64_t s[2]);
void or_dropout_bwd(float *g, const int *mask, long n, float p);
void or_spmm_fwd(int m, const int *indptr, const int *indices, const float *a, const float *b,
                 float *c, int p);
void or_spmm_bwd(int m, int n, const int *indptr, const int *indices, const float *a,
                 float *bgrad, const float *cgrad, int p);
float or_graph_coef(const int *indptr, int src, int dst);
void or_graphsum(int n, const int *indptr, const int *indices, const float *in, float *out,
                 int dim);
void or_relu_fwd(float *x, unsigned char *mask, long n, int training);
void or_relu_bwd(float *g, const unsigned char *mask, long n);
void or_matmul_fwd(const float *a, const float *b, float *c, int m, int n, int p);
void or_matmul_bwd(const float *a, float *agrad, const float *b, float *bgrad,
                   const float *cgrad, int m, int n, int p);
float or_xent_fwd(float *logits, float *grad, const int *truth, int n, int c, int training);
float or_accuracy(const float *logits, const int *truth, int n, int c);
float or_l2_penalty(const float *w, long n, float wd);
float or_adam_step_size(float lr, float beta1, float beta2, int t);
void or_adam_update(float *w, const float *g, float *m, float *v, long n, float step_size,
                    float beta1, float beta2, float eps, float wd, int decay);

/* ---- whole model (hpdga-spring23/src/gcn.cpp:64-274, generalised to L layers the way
 *      src/gcn.cu:47-142 generalises it; L = 2 is exactly the reference) ---- */
typedef struct {
  int num_nodes, input_dim, output_dim, n_layers;
  int hidden_dims[OR_MAX_LAYERS]; /* n_layers - 1 entries */
  float dropouts[OR_MAX_LAYERS];  /* n_layers entries */
  float lr, weight_decay, beta1, beta2, eps;
  unsigned seed; /* 0: hpdga's unseeded rand(); else srand(seed) before init_rand_state */
} or_params;

typedef struct or_gcn or_gcn;

/* Copies the data. label/split: num_nodes ints. Graph CSR includes the implicit self loop
 * exactly as hpdga-spring23/src/parser.cpp:18-48 builds it. */
or_gcn *or_gcn_create(const or_params *p, const int *g_indptr, const int *g_indices,
                      const int *f_indptr, const int *f_indices, const float *f_values,
                      const int *label, const int *split);
void or_gcn_free(or_gcn *g);
void or_gcn_train_epoch(or_gcn *g, float out2[2]);
void or_gcn_eval(or_gcn *g, int split, float out2[2]);
/* forward only (training flag as in Module::forward); leaves loss in *loss_out */
void or_gcn_forward(or_gcn *g, int split, int training, float *loss_out);
int or_gcn_num_vars(const or_gcn *g);
/* which: 0 data, 1 grad. Returns element count; copies into dst if non-null. */
long or_gcn_get_var(const or_gcn *g, int idx, int which, float *dst);
void or_gcn_set_var(or_gcn *g, int idx, const float *src);
void or_gcn_rng_state(const or_gcn *g, uint64_t s2[2]);

#ifdef __cplusplus
}
#endif
#endif
