/* oracle/pgcn_oracle.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * Plain-C restatement of the reference's sequential CPU GCN.  Every function names the
 * reference lines it restates.  The casts spell out the C++ usual arithmetic conversions
 * the reference relies on (float vs double temporaries), so that this file rounds exactly
 * where the reference rounds.  Pinned bit-for-bit against the reference's own build
 * (oracle/_ref) by tests/test_oracle_pinned.py.
 *
 * Build: gcc -O2 -ffp-contract=off (oracle/Makefile).  x86-64 gcc emits no FMA without
 * -mfma, like the reference's own -O3 -std=c++11 build (hpdga-spring23/Makefile:1-3).
 */
#define _DEFAULT_SOURCE /* initstate_r / random_r (glibc) */
#include "pgcn_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------ */
/* RNG                                                                                    */
/* ------------------------------------------------------------------------------------ */

/* hpdga-spring23/src/rand.cpp:6-14: x = rand(), y = rand() from an unseeded glibc rand()
 * (== srand(1)); the first two values of that sequence are 1804289383 and 846930886. */
void or_rng_seed(uint64_t s[2]) {
  s[0] = 1804289383u;
  s[1] = 846930886u;
}

/* The same two draws after srand(seed) (the PART2 `seed` parameter, src/parser.cpp:234):
 * glibc's rand() is random() on a TYPE_3 (128-byte) state, reproduced here on a private
 * state so the process's own rand() is untouched.  seed 0 and 1 give the unseeded values. */
void or_rng_seed_glibc(unsigned seed, uint64_t s[2]) {
  char buf[128];
  struct random_data rd;
  int32_t x = 0, y = 0;
  memset(&rd, 0, sizeof(rd));
  initstate_r(seed, buf, sizeof(buf), &rd);
  random_r(&rd, &x);
  random_r(&rd, &y);
  s[0] = (uint32_t)x;
  s[1] = (uint32_t)y;
}

/* hpdga-spring23/src/rand.cpp:17-28 */
uint32_t or_rng_next(uint64_t s[2]) {
  uint64_t t = s[0];
  const uint64_t u = s[1];
  s[0] = u;
  t ^= t << 23;
  t ^= t >> 17;
  t ^= u ^ (u >> 26);
  s[1] = t;
  return (uint32_t)(t + u) & 0x7fffffffu;
}

/* ------------------------------------------------------------------------------------ */
/* Ops                                                                                    */
/* ------------------------------------------------------------------------------------ */

/* hpdga-spring23/src/variable.cpp:15-19.
 * range = sqrtf(6.0f / (in+out)) in float; element = (float(RAND())/MY_RAND_MAX - 0.5)
 * * range * 2 where float/int divides in float and the rest is evaluated in double. */
void or_glorot(float *w, long n, int in_size, int out_size, uint64_t s[2]) {
  float range = sqrtf(6.0f / (float)(in_size + out_size));
  for (long i = 0; i < n; i++) {
    float r = (float)or_rng_next(s) / (float)OR_RAND_MAX;
    w[i] = (float)((((double)r - 0.5) * (double)range) * 2.0);
  }
}

/* hpdga-spring23/src/module.cpp:208-219: threshold = int(p * MY_RAND_MAX) computed in
 * float; scale = 1 / (1 - p) in float; one RAND() per element, consumed even when the
 * variable keeps no mask (the input). */
void or_dropout_fwd(float *x, int *mask, long n, float p, uint64_t s[2]) {
  const int threshold = (int)(p * (float)OR_RAND_MAX);
  const float scale = 1.0f / (1.0f - p);
  for (long i = 0; i < n; i++) {
    int keep = (int)or_rng_next(s) >= threshold;
    x[i] *= keep ? scale : 0.0f;
    if (mask) mask[i] = keep;
  }
}

/* hpdga-spring23/src/module.cpp:221-228 */
void or_dropout_bwd(float *g, const int *mask, long n, float p) {
  if (!mask) return;
  const float scale = 1.0f / (1.0f - p);
  for (long i = 0; i < n; i++) g[i] *= mask[i] ? scale : 0.0f;
}

/* hpdga-spring23/src/module.cpp:49-59: c = A(CSR) * B, accumulated per output element in
 * CSR order. */
void or_spmm_fwd(int m, const int *indptr, const int *indices, const float *a, const float *b,
                 float *c, int p) {
  memset(c, 0, sizeof(float) * (size_t)m * (size_t)p);
  for (int i = 0; i < m; i++)
    for (int jj = indptr[i]; jj < indptr[i + 1]; jj++) {
      const int j = indices[jj];
      for (int k = 0; k < p; k++) c[(long)i * p + k] += a[jj] * b[(long)j * p + k];
    }
}

/* hpdga-spring23/src/module.cpp:61-72: b.grad = A^T c.grad, scatter-added row by row. */
void or_spmm_bwd(int m, int n, const int *indptr, const int *indices, const float *a,
                 float *bgrad, const float *cgrad, int p) {
  memset(bgrad, 0, sizeof(float) * (size_t)n * (size_t)p);
  for (int i = 0; i < m; i++)
    for (int jj = indptr[i]; jj < indptr[i + 1]; jj++) {
      const int j = indices[jj];
      for (int k = 0; k < p; k++) bgrad[(long)j * p + k] += cgrad[(long)i * p + k] * a[jj];
    }
}

/* hpdga-spring23/src/module.cpp:88-90: coef = 1.0 / sqrtf(int deg_src * int deg_dst):
 * the int product is converted to float for sqrtf, the division is in double and the
 * result is stored to float.  (The GPU reference precomputes the same expression in
 * src/parser.cpp:164-181.) */
float or_graph_coef(const int *indptr, int src, int dst) {
  const int ds = indptr[src + 1] - indptr[src];
  const int dd = indptr[dst + 1] - indptr[dst];
  return (float)(1.0 / (double)sqrtf((float)(ds * dd)));
}

/* hpdga-spring23/src/module.cpp:82-96 (forward) and :98-111 (backward, the same gather
 * applied to grads). */
void or_graphsum(int n, const int *indptr, const int *indices, const float *in, float *out,
                 int dim) {
  memset(out, 0, sizeof(float) * (size_t)n * (size_t)dim);
  for (int src = 0; src < n; src++)
    for (int i = indptr[src]; i < indptr[src + 1]; i++) {
      const int dst = indices[i];
      const float coef = or_graph_coef(indptr, src, dst);
      for (int j = 0; j < dim; j++) out[(long)src * dim + j] += coef * in[(long)dst * dim + j];
    }
}

/* hpdga-spring23/src/module.cpp:173-188 */
void or_relu_fwd(float *x, unsigned char *mask, long n, int training) {
  for (long i = 0; i < n; i++) {
    const int keep = x[i] > 0;
    if (training) mask[i] = (unsigned char)keep;
    if (!keep) x[i] = 0;
  }
}
void or_relu_bwd(float *g, const unsigned char *mask, long n) {
  for (long i = 0; i < n; i++)
    if (!mask[i]) g[i] = 0;
}

/* hpdga-spring23/src/module.cpp:13-22: loop order i, j, k. */
void or_matmul_fwd(const float *a, const float *b, float *c, int m, int n, int p) {
  memset(c, 0, sizeof(float) * (size_t)m * (size_t)p);
  for (int i = 0; i < m; i++)
    for (int j = 0; j < n; j++)
      for (int k = 0; k < p; k++) c[(long)i * p + k] += a[(long)i * n + j] * b[(long)j * p + k];
}

/* hpdga-spring23/src/module.cpp:24-38 */
void or_matmul_bwd(const float *a, float *agrad, const float *b, float *bgrad,
                   const float *cgrad, int m, int n, int p) {
  memset(agrad, 0, sizeof(float) * (size_t)m * (size_t)n);
  memset(bgrad, 0, sizeof(float) * (size_t)n * (size_t)p);
  for (int i = 0; i < m; i++)
    for (int j = 0; j < n; j++) {
      float tmp = 0;
      for (int k = 0; k < p; k++) {
        tmp += cgrad[(long)i * p + k] * b[(long)j * p + k];
        bgrad[(long)j * p + k] += cgrad[(long)i * p + k] * a[(long)i * n + j];
      }
      agrad[(long)i * n + j] = tmp;
    }
}

/* hpdga-spring23/src/module.cpp:122-153.  Logits of labelled rows are max-shifted in
 * place; grad = softmax with 1.0 subtracted at the truth (double temporary), then every
 * grad entry divided by the labelled count. Returns the mean loss. */
float or_xent_fwd(float *logits, float *grad, const int *truth, int n, int c, int training) {
  float total_loss = 0;
  int count = 0;
  if (training) memset(grad, 0, sizeof(float) * (size_t)n * (size_t)c);
  for (int i = 0; i < n; i++) {
    if (truth[i] < 0) continue;
    count++;
    float *logit = &logits[(long)i * c];
    float max_logit = (float)-1e30, sum_exp = 0;
    for (int j = 0; j < c; j++) max_logit = fmaxf(max_logit, logit[j]);
    for (int j = 0; j < c; j++) {
      logit[j] -= max_logit;
      sum_exp += expf(logit[j]);
    }
    total_loss += logf(sum_exp) - logit[truth[i]];
    if (training) {
      for (int j = 0; j < c; j++) {
        float prob = expf(logit[j]) / sum_exp;
        grad[(long)i * c + j] = prob;
      }
      grad[(long)i * c + truth[i]] = (float)((double)grad[(long)i * c + truth[i]] - 1.0);
    }
  }
  float loss = total_loss / (float)count;
  if (training)
    for (long i = 0; i < (long)n * c; i++) grad[i] /= (float)count;
  return loss;
}

/* hpdga-spring23/src/gcn.cpp:150-164: a row is wrong if any logit is strictly greater
 * than the truth logit. */
float or_accuracy(const float *logits, const int *truth, int n, int c) {
  int wrong = 0, total = 0;
  for (int i = 0; i < n; i++) {
    if (truth[i] < 0) continue;
    total++;
    const float t = logits[(long)i * c + truth[i]];
    for (int j = 0; j < c; j++)
      if (logits[(long)i * c + j] > t) {
        wrong++;
        break;
      }
  }
  return (float)(total - wrong) / (float)total;
}

/* hpdga-spring23/src/gcn.cpp:167-174: sequential float sum of squares of W1 only. */
float or_l2_penalty(const float *w, long n, float wd) {
  float l2 = 0;
  for (long i = 0; i < n; i++) {
    const float x = w[i];
    l2 += x * x;
  }
  return wd * l2 / 2.0f;
}

/* hpdga-spring23/src/optim.cpp:24 */
float or_adam_step_size(float lr, float beta1, float beta2, int t) {
  return lr * sqrtf(1.0f - powf(beta2, (float)t)) / (1.0f - powf(beta1, (float)t));
}

/* hpdga-spring23/src/optim.cpp:25-33: the (1.0 - beta) terms are double, beta * m is a
 * float product promoted to double, m and v are stored as float. */
void or_adam_update(float *w, const float *g, float *m, float *v, long n, float step_size,
                    float beta1, float beta2, float eps, float wd, int decay) {
  for (long i = 0; i < n; i++) {
    float grad = g[i];
    if (decay) grad += wd * w[i];
    m[i] = (float)((double)(beta1 * m[i]) + (1.0 - (double)beta1) * (double)grad);
    v[i] = (float)((double)(beta2 * v[i]) + ((1.0 - (double)beta2) * (double)grad) * (double)grad);
    w[i] -= step_size * m[i] / (sqrtf(v[i]) + eps);
  }
}

/* ------------------------------------------------------------------------------------ */
/* Model                                                                                  */
/* ------------------------------------------------------------------------------------ */

typedef struct {
  float *data, *grad; /* grad NULL when the variable has no grad (the input) */
  long size;
} or_var;

enum { M_DROPOUT, M_SPMM, M_GRAPHSUM, M_RELU, M_MATMUL, M_XENT };

typedef struct {
  int kind;
  int a, b, c;  /* variable indices (in/out/weight as the kind needs) */
  int m, n, p;  /* dims */
  float drop_p; /* dropout rate */
  int *imask;   /* dropout mask (NULL for the input) */
  unsigned char *bmask; /* relu mask */
} or_module;

struct or_gcn {
  or_params p;
  int n_nodes;
  /* data */
  int *g_indptr, *g_indices, *f_indptr, *f_indices, *label, *split;
  float *f_values;
  long g_nnz, f_nnz;
  /* variables / modules */
  or_var vars[3 * OR_MAX_LAYERS + 1];
  int n_vars;
  or_module mods[4 * OR_MAX_LAYERS];
  int n_mods;
  int weight_idx[OR_MAX_LAYERS];
  /* adam */
  float *adam_m[OR_MAX_LAYERS], *adam_v[OR_MAX_LAYERS];
  int step_count;
  /* state */
  int *truth;
  float loss;
  uint64_t rng[2];
};

static int add_var(or_gcn *g, long size, int requires_grad) {
  or_var *v = &g->vars[g->n_vars];
  v->size = size;
  v->data = (float *)calloc((size_t)size, sizeof(float));
  v->grad = requires_grad ? (float *)calloc((size_t)size, sizeof(float)) : NULL;
  return g->n_vars++;
}

static or_module *add_mod(or_gcn *g, int kind) {
  or_module *m = &g->mods[g->n_mods++];
  memset(m, 0, sizeof *m);
  m->kind = kind;
  return m;
}

static void add_dropout(or_gcn *g, int var, float p) {
  or_module *m = add_mod(g, M_DROPOUT);
  m->a = var;
  m->drop_p = p;
  /* hpdga-spring23/src/module.cpp:196-202: mask only when the variable has a grad */
  m->imask = g->vars[var].grad ? (int *)calloc((size_t)g->vars[var].size, sizeof(int)) : NULL;
}

/* hpdga-spring23/src/gcn.cpp:64-128 (2 layers); L layers follow src/gcn.cu:47-142. */
or_gcn *or_gcn_create(const or_params *p, const int *g_indptr, const int *g_indices,
                      const int *f_indptr, const int *f_indices, const float *f_values,
                      const int *label, const int *split) {
  or_gcn *g = (or_gcn *)calloc(1, sizeof(or_gcn));
  g->p = *p;
  const int N = p->num_nodes, L = p->n_layers;
  g->n_nodes = N;
  g->g_nnz = g_indptr[N];
  g->f_nnz = f_indptr[N];
#define DUP(dst, src, cnt, T)                              \
  do {                                                     \
    dst = (T *)malloc(sizeof(T) * (size_t)((cnt) + 1));    \
    memcpy(dst, src, sizeof(T) * (size_t)(cnt));           \
  } while (0)
  DUP(g->g_indptr, g_indptr, N + 1, int);
  DUP(g->g_indices, g_indices, g->g_nnz, int);
  DUP(g->f_indptr, f_indptr, N + 1, int);
  DUP(g->f_indices, f_indices, g->f_nnz, int);
  DUP(g->f_values, f_values, g->f_nnz, float);
  DUP(g->label, label, N, int);
  DUP(g->split, split, N, int);
#undef DUP
  g->truth = (int *)calloc((size_t)N, sizeof(int));
  if (p->seed) /* init_rand_state(), gcn.cpp:65 */
    or_rng_seed_glibc(p->seed, g->rng);
  else
    or_rng_seed(g->rng);

  int dims[OR_MAX_LAYERS + 1];
  dims[0] = p->input_dim;
  for (int l = 1; l < L; l++) dims[l] = p->hidden_dims[l - 1];
  dims[L] = p->output_dim;

  /* input (no grad) */
  int input = add_var(g, g->f_nnz, 0);
  add_dropout(g, input, p->dropouts[0]);
  int prev = -1;
  for (int l = 0; l < L; l++) {
    const int din = dims[l], dout = dims[l + 1];
    if (l > 0) add_dropout(g, prev, p->dropouts[l]);
    int var1 = add_var(g, (long)N * dout, 1);
    int w = add_var(g, (long)din * dout, 1);
    g->weight_idx[l] = w;
    /* glorot right after the weight is created, gcn.cpp:78-79 / :96-97 */
    or_glorot(g->vars[w].data, g->vars[w].size, din, dout, g->rng);
    or_module *mm = add_mod(g, l == 0 ? M_SPMM : M_MATMUL);
    mm->a = l == 0 ? input : prev;
    mm->b = w;
    mm->c = var1;
    mm->m = N;
    mm->n = din;
    mm->p = dout;
    int var2 = add_var(g, (long)N * dout, 1);
    or_module *gs = add_mod(g, M_GRAPHSUM);
    gs->a = var1;
    gs->b = var2;
    gs->p = dout;
    if (l < L - 1) {
      or_module *r = add_mod(g, M_RELU);
      r->a = var2;
      r->bmask = (unsigned char *)calloc((size_t)N * dout, 1);
    } else {
      or_module *x = add_mod(g, M_XENT);
      x->a = var2;
      x->p = dout;
    }
    prev = var2;
  }
  for (int l = 0; l < L; l++) {
    long sz = g->vars[g->weight_idx[l]].size;
    g->adam_m[l] = (float *)calloc((size_t)sz, sizeof(float));
    g->adam_v[l] = (float *)calloc((size_t)sz, sizeof(float));
  }
  return g;
}

void or_gcn_free(or_gcn *g) {
  if (!g) return;
  for (int i = 0; i < g->n_vars; i++) {
    free(g->vars[i].data);
    free(g->vars[i].grad);
  }
  for (int i = 0; i < g->n_mods; i++) {
    free(g->mods[i].imask);
    free(g->mods[i].bmask);
  }
  for (int l = 0; l < g->p.n_layers; l++) {
    free(g->adam_m[l]);
    free(g->adam_v[l]);
  }
  free(g->g_indptr);
  free(g->g_indices);
  free(g->f_indptr);
  free(g->f_indices);
  free(g->f_values);
  free(g->label);
  free(g->split);
  free(g->truth);
  free(g);
}

static void mod_forward(or_gcn *g, or_module *m, int training) {
  const int N = g->n_nodes;
  or_var *v = g->vars;
  switch (m->kind) {
    case M_DROPOUT:
      if (!training) return; /* module.cpp:209 */
      or_dropout_fwd(v[m->a].data, m->imask, v[m->a].size, m->drop_p, g->rng);
      break;
    case M_SPMM:
      or_spmm_fwd(N, g->f_indptr, g->f_indices, v[m->a].data, v[m->b].data, v[m->c].data, m->p);
      break;
    case M_GRAPHSUM:
      or_graphsum(N, g->g_indptr, g->g_indices, v[m->a].data, v[m->b].data, m->p);
      break;
    case M_RELU:
      or_relu_fwd(v[m->a].data, m->bmask, v[m->a].size, training);
      break;
    case M_MATMUL:
      or_matmul_fwd(v[m->a].data, v[m->b].data, v[m->c].data, m->m, m->n, m->p);
      break;
    case M_XENT:
      g->loss = or_xent_fwd(v[m->a].data, v[m->a].grad, g->truth, N, m->p, training);
      break;
  }
}

static void mod_backward(or_gcn *g, or_module *m) {
  const int N = g->n_nodes;
  or_var *v = g->vars;
  switch (m->kind) {
    case M_DROPOUT:
      or_dropout_bwd(v[m->a].grad, m->imask, v[m->a].size, m->drop_p);
      break;
    case M_SPMM:
      or_spmm_bwd(N, m->n, g->f_indptr, g->f_indices, v[m->a].data, v[m->b].grad, v[m->c].grad,
                  m->p);
      break;
    case M_GRAPHSUM:
      or_graphsum(N, g->g_indptr, g->g_indices, v[m->b].grad, v[m->a].grad, m->p);
      break;
    case M_RELU:
      or_relu_bwd(v[m->a].grad, m->bmask, v[m->a].size);
      break;
    case M_MATMUL:
      or_matmul_bwd(v[m->a].data, v[m->a].grad, v[m->b].data, v[m->b].grad, v[m->c].grad, m->m,
                    m->n, m->p);
      break;
    case M_XENT:
      break; /* module.cpp:155-156 */
  }
}

/* gcn.cpp:136-147 */
static void set_input_truth(or_gcn *g, int split) {
  memcpy(g->vars[0].data, g->f_values, sizeof(float) * (size_t)g->f_nnz);
  for (int i = 0; i < g->n_nodes; i++) g->truth[i] = g->split[i] == split ? g->label[i] : -1;
}

static float l2_of_w1(or_gcn *g) {
  const or_var *w1 = &g->vars[g->weight_idx[0]];
  return or_l2_penalty(w1->data, w1->size, g->p.weight_decay);
}

static float acc_of_output(or_gcn *g) {
  return or_accuracy(g->vars[g->n_vars - 1].data, g->truth, g->n_nodes, g->p.output_dim);
}

void or_gcn_forward(or_gcn *g, int split, int training, float *loss_out) {
  set_input_truth(g, split);
  for (int i = 0; i < g->n_mods; i++) mod_forward(g, &g->mods[i], training);
  if (loss_out) *loss_out = g->loss;
}

/* gcn.cpp:179-198 */
void or_gcn_train_epoch(or_gcn *g, float out2[2]) {
  or_gcn_forward(g, 1, 1, NULL);
  out2[0] = g->loss + l2_of_w1(g);
  out2[1] = acc_of_output(g);
  for (int i = g->n_mods - 1; i >= 0; i--) mod_backward(g, &g->mods[i]);
  /* Adam::step, optim.cpp:23-35; decay only for W1 (gcn.cpp:127) */
  g->step_count++;
  const float ss = or_adam_step_size(g->p.lr, g->p.beta1, g->p.beta2, g->step_count);
  for (int l = 0; l < g->p.n_layers; l++) {
    or_var *w = &g->vars[g->weight_idx[l]];
    or_adam_update(w->data, w->grad, g->adam_m[l], g->adam_v[l], w->size, ss, g->p.beta1,
                   g->p.beta2, g->p.eps, g->p.weight_decay, l == 0);
  }
}

/* gcn.cpp:204-212 */
void or_gcn_eval(or_gcn *g, int split, float out2[2]) {
  or_gcn_forward(g, split, 0, NULL);
  out2[0] = g->loss + l2_of_w1(g);
  out2[1] = acc_of_output(g);
}

int or_gcn_num_vars(const or_gcn *g) { return g->n_vars; }

long or_gcn_get_var(const or_gcn *g, int idx, int which, float *dst) {
  if (idx < 0 || idx >= g->n_vars) return -1;
  const or_var *v = &g->vars[idx];
  const float *src = which ? v->grad : v->data;
  if (!src) return 0;
  if (dst) memcpy(dst, src, sizeof(float) * (size_t)v->size);
  return v->size;
}

void or_gcn_set_var(or_gcn *g, int idx, const float *src) {
  or_var *v = &g->vars[idx];
  memcpy(v->data, src, sizeof(float) * (size_t)v->size);
}

void or_gcn_rng_state(const or_gcn *g, uint64_t s2[2]) {
  s2[0] = g->rng[0];
  s2[1] = g->rng[1];
}
