// parallel-gcn_amd/csrc/host/data.hpp -- host-side graph data and the kept hpdga loader.
//
// SparseIndex / GCNData mirror include/sparse.cuh:11-17 and include/gcn.cuh:51-58 (and
// hpdga-spring23/include/sparse.h:12-17, gcn.h:18-24). Parser keeps the hpdga loader's API
// and semantics (hpdga-spring23/include/parser.h:10-24, src/parser.cpp:6-140): implicit
// self loop first, neighbours in file order, duplicates kept, an unterminated last line
// dropped, empty svmlight lines give label -1, input_dim = max feature id + 1,
// output_dim = max label + 1.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace pgcn {

struct SparseIndex {
  std::vector<int> indices;
  std::vector<int> indptr;
};

struct GCNData {
  SparseIndex feature_index, graph;
  std::vector<int> split;
  std::vector<int> label;
  std::vector<float> feature_value;
  int num_nodes = 0, input_dim = 0, output_dim = 0;
};

class Parser {
 public:
  // Opens <root>/data/<name>.{graph,split,svmlight} (the reference opens data/<name>.*
  // relative to the working directory; root "." reproduces that).
  Parser(GCNData *data, const std::string &name, const std::string &root = ".");
  bool parse();

 private:
  GCNData *data_;
  std::string graph_path_, split_path_, svm_path_;
};

// Seeded reddit-shaped synthetic dataset: Chung-Lu power-law graph
// (Pareto alpha 1.8 weights capped at 40x mean, no self loops before the loader's implicit
// ones, neighbours sorted), dense N(0,1) features quantised to 4 decimals, uniform labels,
// split sizes scaled from reddit's 153,431 / 23,831 / 55,703.
void make_synthetic(GCNData *d, int n, int f, int c, long long undirected_edges,
                    uint64_t seed);

// Binary dataset cache: the parsed arrays of GCNData as one file
// ("PGCNDS01" header, sizes, the source files' size + mtime stamps, raw little-endian arrays,
// FNV-1a 64 checksum of the payload).  load_binary fails (returns false) on a missing file,
// another version, stamps that differ from `stamps` (when given), a short file or a checksum
// mismatch; the caller then parses the text.
struct FileStamp {
  long long size = -1, mtime_ns = -1;
};
bool stamp_file(const std::string &path, FileStamp *st);
bool save_binary(const GCNData &d, const std::string &path, const FileStamp stamps[3]);
bool load_binary(GCNData *d, const std::string &path, const FileStamp *stamps);
// Parser + cache: <root>/data/<name>.pgcnbin is read when its stamps match the three text
// files, else the text is parsed and the cache (re)written (best effort).  *from_cache tells
// which happened.
bool load_dataset_cached(GCNData *d, const std::string &root, const std::string &name,
                         bool *from_cache);

// True when every row lists all features 0..F-1 in order (a dense matrix in CSR form).
bool features_dense(const GCNData &d);

}  // namespace pgcn
