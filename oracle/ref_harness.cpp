// oracle/ref_harness.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never measured as product).
//
// Drives the reference's own sequential CPU GCN (hpdga-spring23/src/*.cpp, compiled from
// where they lie under /root/reference by oracle/Makefile; no reference source is copied
// into this repository).  Two roles:
//
//   1. `ref_golden` CLI: parses a reference dataset with the reference Parser
//      (hpdga-spring23/src/parser.cpp:6-140), builds the reference GCN
//      (hpdga-spring23/src/gcn.cpp:64-128) and dumps golden tensors / epoch lines that pin
//      the C restatement in oracle/pgcn_oracle.c and the HIP path.
//   2. `libhpdga_ref.so`: a tiny C ABI around the same objects, fed from in-memory arrays
//      (no text parse), used by tests and by bench.py's `cpu_baseline` leg
//      ("kind": "reference") to time the reference's own sequential epoch.
//
// Private members of GCN are reached with the `#define private public` trick documented in
// SURVEY.md §7 step 2; all standard headers are included first so the macros only touch
// the reference headers.
#include <sstream>
#include <iostream>
#include <fstream>
#include <vector>
#include <utility>
#include <string>
#include <cmath>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cstdint>
#include <tuple>
#include <unistd.h>
#include <sys/stat.h>

#define class struct
#define private public
#include "gcn.h"
#include "parser.h"
#include "rand.h"
#include "timer.h"
#undef private
#undef class

namespace {

void dump(const std::string &dir, const std::string &name, const void *p, size_t bytes) {
  std::string path = dir + "/" + name + ".bin";
  FILE *f = fopen(path.c_str(), "wb");
  if (!f) { perror(path.c_str()); exit(2); }
  if (bytes) fwrite(p, 1, bytes, f);
  fclose(f);
}
void dumpf(const std::string &dir, const std::string &name, const std::vector<float> &v) {
  dump(dir, name, v.data(), v.size() * sizeof(float));
}
void dumpi(const std::string &dir, const std::string &name, const std::vector<int> &v) {
  dump(dir, name, v.data(), v.size() * sizeof(int));
}
void dump_state(const std::string &dir, const std::string &name) {
  dump(dir, name, rand_state, sizeof(rand_state));
}

// Module order fixed by hpdga-spring23/src/gcn.cpp:70-119:
// 0 Dropout(input) 1 SparseMatmul 2 GraphSum 3 ReLU 4 Dropout(l1_var2) 5 Matmul 6 GraphSum 7 CE
// Variable order: 0 input 1 l1_var1 2 W1 3 l1_var2 4 l2_var1 5 W2 6 output
const char *kVarNames[7] = {"input", "l1_var1", "W1", "l1_var2", "l2_var1", "W2", "output"};

void dump_vars(GCN &g, const std::string &dir, const std::string &tag, bool grads) {
  for (int i = 0; i < 7; i++) {
    dumpf(dir, tag + "_" + kVarNames[i], g.variables[i].data);
    if (grads && !g.variables[i].grad.empty())
      dumpf(dir, tag + "_" + kVarNames[i] + "_grad", g.variables[i].grad);
  }
}

int golden_main(int argc, char **argv) {
  // ref_golden <reference_dir_containing_data/> <dataset> <outdir> [epochs]
  if (argc < 4) {
    fprintf(stderr, "usage: ref_golden <dir-with-data/> <dataset> <outdir> [epochs]\n");
    return 1;
  }
  std::string root = argv[1], name = argv[2], out = argv[3];
  int epochs = argc > 4 ? atoi(argv[4]) : 100;
  mkdir(out.c_str(), 0755);
  char cwd[4096];
  if (!getcwd(cwd, sizeof cwd)) return 2;
  std::string outabs = out[0] == '/' ? out : std::string(cwd) + "/" + out;
  if (chdir(root.c_str()) != 0) { perror("chdir"); return 2; }

  GCNParams params = GCNParams::get_default();
  GCNData data;
  Parser parser(&params, &data, name);
  if (!parser.parse()) { fprintf(stderr, "Cannot read input: %s\n", name.c_str()); return 3; }
  params.epochs = epochs;
  out = outabs;

  // parsed CSR (pins the loader, a1-a3)
  dumpi(out, "graph_indptr", data.graph.indptr);
  dumpi(out, "graph_indices", data.graph.indices);
  dumpi(out, "feat_indptr", data.feature_index.indptr);
  dumpi(out, "feat_indices", data.feature_index.indices);
  dumpf(out, "feat_values", data.feature_value);
  dumpi(out, "label", data.label);
  dumpi(out, "split", data.split);
  int dims[4] = {params.num_nodes, params.input_dim, params.hidden_dim, params.output_dim};
  dump(out, "dims", dims, sizeof dims);

  // first 64 raw xorshift draws from the default seed state (a5)
  {
    init_rand_state();
    uint64_t s0[2] = {rand_state[0], rand_state[1]};
    dump(out, "rng_seed_state", s0, sizeof s0);
    std::vector<int> draws(64);
    for (auto &d : draws) d = (int)RAND();
    dumpi(out, "rng_first64", draws);
  }
  // init_rand_state() draws from glibc rand(); restore the fresh-process sequence
  // (unseeded rand() == srand(1)) so the GCN below sees the same seed as gcn-seq does.
  srand(1);

  GCN gcn(params, &data);  // re-inits rand_state (hpdga-spring23/src/gcn.cpp:65)
  dump_state(out, "rng_after_ctor");
  dump_vars(gcn, out, "init", false);

  // Epoch 1, step by step (same sequence as GCN::train_epoch, gcn.cpp:179-198).
  gcn.set_input();
  gcn.set_truth(1);
  for (auto m : gcn.modules) m->forward(true);
  dump_state(out, "rng_after_e1_fwd");
  float train_loss = gcn.loss + gcn.get_l2_penalty();
  float train_acc = gcn.get_accuracy();
  for (int i = (int)gcn.modules.size() - 1; i >= 0; i--) gcn.modules[i]->backward();
  dump_vars(gcn, out, "e1", true);
  gcn.optimizer.step();
  dumpf(out, "e1_W1_after_step", gcn.variables[2].data);
  dumpf(out, "e1_W2_after_step", gcn.variables[5].data);
  {
    float s[2] = {train_loss, train_acc};
    dump(out, "e1_train_scalars", s, sizeof s);
  }
  float val_loss, val_acc;
  std::tie(val_loss, val_acc) = gcn.eval(2);
  dumpf(out, "e1_eval_logits", gcn.variables[6].data);
  {
    float s[2] = {val_loss, val_acc};
    dump(out, "e1_eval_scalars", s, sizeof s);
  }
  dump_state(out, "rng_after_e1");

  // Remaining epochs via the reference's own methods; record every epoch line.
  std::vector<float> lines;
  lines.insert(lines.end(), {train_loss, train_acc, val_loss, val_acc});
  for (int e = 2; e <= epochs; e++) {
    float a, b, c, d;
    std::tie(a, b) = gcn.train_epoch();
    std::tie(c, d) = gcn.eval(2);
    lines.insert(lines.end(), {a, b, c, d});
  }
  dumpf(out, "epoch_lines", lines);
  dumpf(out, "final_W1", gcn.variables[2].data);
  dumpf(out, "final_W2", gcn.variables[5].data);
  dumpf(out, "final_eval_logits", gcn.variables[6].data);
  float tl, ta;
  std::tie(tl, ta) = gcn.eval(3);
  float t[2] = {tl, ta};
  dump(out, "test_scalars", t, sizeof t);
  dumpf(out, "final_test_logits", gcn.variables[6].data);
  // printed form, as hpdga-spring23/src/gcn.cpp:229-232 prints it (time field omitted)
  std::string txt = out + "/epoch_lines.txt";
  FILE *f = fopen(txt.c_str(), "w");
  for (int e = 0; e < epochs; e++)
    fprintf(f, "epoch=%d train_loss=%.5f train_acc=%.5f val_loss=%.5f val_acc=%.5f\n", e + 1,
            lines[4 * e], lines[4 * e + 1], lines[4 * e + 2], lines[4 * e + 3]);
  fprintf(f, "test_loss=%.5f test_acc=%.5f\n", tl, ta);
  fclose(f);
  return 0;
}

}  // namespace

// ---------------------------------------------------------------------------------------
// C ABI for ctypes (tests + bench cpu_baseline). In-memory data, no text parse.
extern "C" {

struct RefHandle {
  GCNData data;
  GCN *gcn;
};

void *ref_create(int num_nodes, int input_dim, int hidden_dim, int output_dim, float dropout,
                 float lr, float wd, int epochs, const int *g_indptr, const int *g_indices,
                 long long g_nnz, const int *f_indptr, const int *f_indices, const float *f_values,
                 long long f_nnz, const int *label, const int *split) {
  RefHandle *h = new RefHandle();
  h->data.graph.indptr.assign(g_indptr, g_indptr + num_nodes + 1);
  h->data.graph.indices.assign(g_indices, g_indices + g_nnz);
  h->data.feature_index.indptr.assign(f_indptr, f_indptr + num_nodes + 1);
  h->data.feature_index.indices.assign(f_indices, f_indices + f_nnz);
  h->data.feature_value.assign(f_values, f_values + f_nnz);
  h->data.label.assign(label, label + num_nodes);
  h->data.split.assign(split, split + num_nodes);
  GCNParams p = GCNParams::get_default();
  p.num_nodes = num_nodes;
  p.input_dim = input_dim;
  p.hidden_dim = hidden_dim;
  p.output_dim = output_dim;
  p.dropout = dropout;
  p.learning_rate = lr;
  p.weight_decay = wd;
  p.epochs = epochs;
  p.early_stopping = 0;
  srand(1);  // every handle starts from the fresh-process seed, as gcn-seq does
  h->gcn = new GCN(p, &h->data);
  return h;
}

void ref_train_epoch(void *hp, float *out2) {
  RefHandle *h = (RefHandle *)hp;
  float a, b;
  std::tie(a, b) = h->gcn->train_epoch();
  out2[0] = a;
  out2[1] = b;
}

void ref_eval(void *hp, int split, float *out2) {
  RefHandle *h = (RefHandle *)hp;
  float a, b;
  std::tie(a, b) = h->gcn->eval(split);
  out2[0] = a;
  out2[1] = b;
}

// Copies variable `idx` (0..6, order above) data (which=0) or grad (which=1) to `dst`.
long long ref_get_var(void *hp, int idx, int which, float *dst) {
  RefHandle *h = (RefHandle *)hp;
  const std::vector<float> &v = which ? h->gcn->variables[idx].grad : h->gcn->variables[idx].data;
  if (dst) memcpy(dst, v.data(), v.size() * sizeof(float));
  return (long long)v.size();
}

void ref_rand_state(unsigned long long *s2) {
  s2[0] = rand_state[0];
  s2[1] = rand_state[1];
}

void ref_free(void *hp) {
  RefHandle *h = (RefHandle *)hp;
  delete h->gcn;
  delete h;
}

}  // extern "C"

#ifdef REF_GOLDEN_MAIN
int main(int argc, char **argv) { return golden_main(argc, argv); }
#endif
