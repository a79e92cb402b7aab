// parallel-gcn_amd/csrc/main.cpp -- `gcn-par <dataset> [file=<params>] [root=<dir>] [cache=1]`
// The reference's entry point (src/main.cpp:9-61): parse the dataset with the kept loader,
// build the GCN, run the epochs printing the reference's epoch lines.  Parameters come from
// a key=value file with the reference's keys (parameters/parameters_<ds>.txt layout:
// n_layers, hidden_dims, dropouts, epochs, early_stopping, learning_rate, weight_decay,
// beta1, beta2, eps, seed (srand seed of the xorshift state); the CUDA launch knobs
// num_blocks_factor/num_threads are accepted and ignored) -- our own tiny parser, GetPot is
// not vendored.  no_feature=1 is the PART2 NO_FEATURE build (feature values 1.0).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>

#include "../../include/pgcn.h"

static void trim(std::string &s) {
  size_t a = s.find_first_not_of(" \t\r\n"), b = s.find_last_not_of(" \t\r\n");
  s = a == std::string::npos ? "" : s.substr(a, b - a + 1);
}

static bool load_params(const char *path, pgcn_params *p) {
  std::ifstream f(path);
  if (!f.is_open()) return false;
  std::string line;
  while (std::getline(f, line)) {
    const size_t hash = line.find('#');
    if (hash != std::string::npos) line = line.substr(0, hash);
    const size_t eq = line.find('=');
    if (eq == std::string::npos) continue;
    std::string k = line.substr(0, eq), v = line.substr(eq + 1);
    trim(k);
    trim(v);
    auto list = [&](auto *dst, bool is_float) {
      std::stringstream ss(v);
      std::string tok;
      int n = 0;
      while (std::getline(ss, tok, ',') && n < PGCN_MAX_LAYERS) {
        if (is_float) ((float *)dst)[n++] = std::strtof(tok.c_str(), nullptr);
        else ((int *)dst)[n++] = std::atoi(tok.c_str());
      }
      return n;
    };
    if (k == "n_layers") p->n_layers = std::atoi(v.c_str());
    else if (k == "hidden_dims") list(p->hidden_dims, false);
    else if (k == "dropouts") list(p->dropouts, true);
    else if (k == "epochs") p->epochs = std::atoi(v.c_str());
    else if (k == "early_stopping") p->early_stopping = std::atoi(v.c_str());
    else if (k == "learning_rate") p->learning_rate = std::strtof(v.c_str(), nullptr);
    else if (k == "weight_decay") p->weight_decay = std::strtof(v.c_str(), nullptr);
    else if (k == "beta1") p->beta1 = std::strtof(v.c_str(), nullptr);
    else if (k == "beta2") p->beta2 = std::strtof(v.c_str(), nullptr);
    else if (k == "eps") p->eps = std::strtof(v.c_str(), nullptr);
    else if (k == "seed") p->seed = (unsigned)std::strtoul(v.c_str(), nullptr, 10);
  }
  return true;
}

int main(int argc, char **argv) {
  if (argc < 2) {
    fprintf(stderr, "Give one input file name as argument [cora pubmed citeseer reddit]\n");
    return EXIT_FAILURE;
  }
  const char *name = argv[1];
  std::string root = ".", file;
  bool cache = false;  // cache=1: read/write the binary dataset cache data/<name>.pgcnbin
  bool no_feature = false;  // no_feature=1: the PART2 NO_FEATURE build (feature values 1.0)
  for (int i = 2; i < argc; i++) {
    if (!std::strncmp(argv[i], "file=", 5)) file = argv[i] + 5;
    if (!std::strncmp(argv[i], "root=", 5)) root = argv[i] + 5;
    if (!std::strcmp(argv[i], "cache=1")) cache = true;
    if (!std::strcmp(argv[i], "no_feature=1")) no_feature = true;
  }
  pgcn_params p;
  pgcn_params_default(&p);
  if (!file.empty() && !load_params(file.c_str(), &p)) {
    fprintf(stderr, "cannot read parameter file %s\n", file.c_str());
    return EXIT_FAILURE;
  }
  pgcn_dataset *ds = nullptr;
  const int lst = cache ? pgcn_dataset_load_cached(root.c_str(), name, &ds, nullptr)
                        : pgcn_dataset_load(root.c_str(), name, &ds);
  if (lst != PGCN_OK) {
    fprintf(stderr, "Cannot read input: %s\n", name);
    return EXIT_FAILURE;
  }
  if (no_feature) pgcn_dataset_binarize(ds);
  pgcn_data view;
  pgcn_dataset_view(ds, &view, &p.input_dim, &p.output_dim);
  p.num_nodes = view.num_nodes;
  pgcn_gcn *g = nullptr;
  int st = pgcn_gcn_create(&p, &view, 0, &g);
  if (st != PGCN_OK) {
    fprintf(stderr, "GCN creation failed: %s\n", pgcn_status_string(st));
    return EXIT_FAILURE;
  }
  st = pgcn_gcn_run(g, 1);
  pgcn_gcn_destroy(g);
  pgcn_dataset_free(ds);
  return st == PGCN_OK ? EXIT_SUCCESS : EXIT_FAILURE;
}
