// parallel-gcn_amd/csrc/host/data.cpp -- hpdga loader semantics + synthetic inputs.
#include "data.hpp"

#include <algorithm>
#include <atomic>
#include <cctype>
#include <cerrno>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>

#include <sys/stat.h>

#include "graph.hpp"  // parallel_for

namespace pgcn {

namespace {

bool read_file(const std::string &path, std::string *out) {
  std::ifstream f(path, std::ios::binary);
  if (!f.is_open()) return false;
  std::ostringstream ss;
  ss << f.rdbuf();
  *out = ss.str();
  return true;
}

// Calls fn(begin, end) for every '\n'-terminated line: `getline; if (eof) break` in the
// reference (hpdga parser.cpp:23-27) drops an unterminated last line.
template <class Fn>
void for_each_line(const std::string &buf, Fn fn) {
  size_t pos = 0;
  while (true) {
    const size_t nl = buf.find('\n', pos);
    if (nl == std::string::npos) break;
    fn(buf.data() + pos, buf.data() + nl);
    pos = nl + 1;
  }
}

inline bool is_ws(char c) { return std::isspace((unsigned char)c) != 0; }

// istream >> int on [p, end): skip whitespace, parse; false if no integer (failbit).
bool next_int(const char *&p, const char *end, int *v) {
  while (p < end && is_ws(*p)) p++;
  if (p >= end) return false;
  char tmp[32];
  size_t n = 0;
  const char *q = p;
  if (q < end && (*q == '+' || *q == '-')) tmp[n++] = *q++;
  while (q < end && std::isdigit((unsigned char)*q) && n < sizeof tmp - 1) tmp[n++] = *q++;
  tmp[n] = 0;
  if (n == 0 || !std::isdigit((unsigned char)tmp[n - 1])) return false;
  errno = 0;
  const long x = std::strtol(tmp, nullptr, 10);
  p = q;
  if (errno == ERANGE || x > INT_MAX || x < INT_MIN) return false;
  *v = (int)x;
  return true;
}

}  // namespace

Parser::Parser(GCNData *data, const std::string &name, const std::string &root)
    : data_(data),
      graph_path_(root + "/data/" + name + ".graph"),
      split_path_(root + "/data/" + name + ".split"),
      svm_path_(root + "/data/" + name + ".svmlight") {}

bool Parser::parse() {
  std::string g, s, v;
  // isValidInput(): all three files must open (hpdga parser.cpp:50-53)
  if (!read_file(graph_path_, &g) || !read_file(split_path_, &s) || !read_file(svm_path_, &v))
    return false;
  GCNData &d = *data_;

  // parseGraph (hpdga parser.cpp:18-48)
  d.graph.indptr.assign(1, 0);
  d.graph.indices.clear();
  int node = 0;
  for_each_line(g, [&](const char *p, const char *end) {
    d.graph.indices.push_back(node);  // implicit self connection
    d.graph.indptr.push_back(d.graph.indptr.back() + 1);
    node++;
    int nb;
    while (next_int(p, end, &nb)) {
      d.graph.indices.push_back(nb);
      d.graph.indptr.back() += 1;
    }
  });
  d.num_nodes = node;

  // parseNode (hpdga parser.cpp:59-104)
  d.feature_index.indptr.assign(1, 0);
  d.feature_index.indices.clear();
  d.feature_value.clear();
  d.label.clear();
  int max_idx = 0, max_label = 0;
  for_each_line(v, [&](const char *p, const char *end) {
    d.feature_index.indptr.push_back(d.feature_index.indptr.back());
    const char *q = p;
    while (q < end && is_ws(*q)) q++;
    if (q >= end) {  // nothing to extract: the sentry fails, label keeps its -1
      d.label.push_back(-1);
      return;
    }
    int label;
    if (!next_int(p, end, &label)) {  // a non-number: num_get stores 0 and fails
      d.label.push_back(0);
      return;
    }
    d.label.push_back(label);
    max_label = std::max(max_label, label);
    // "k:v" tokens
    while (true) {
      while (p < end && is_ws(*p)) p++;
      if (p >= end) break;
      const char *tok = p;
      while (p < end && !is_ws(*p)) p++;
      const char *tend = p;
      int k = 0;
      const char *t = tok;
      next_int(t, tend, &k);
      if (t < tend) t++;  // the ':' (kv_ss >> col)
      char num[64];
      size_t n = std::min((size_t)(tend - t), sizeof num - 1);
      std::memcpy(num, t, n);
      num[n] = 0;
      const float val = std::strtof(num, nullptr);
      d.feature_value.push_back(val);
      d.feature_index.indices.push_back(k);
      d.feature_index.indptr.back() += 1;
      max_idx = std::max(max_idx, k);
    }
  });
  d.input_dim = max_idx + 1;
  d.output_dim = max_label + 1;

  // parseSplit (hpdga parser.cpp:106-116): std::stoi per line
  d.split.clear();
  bool ok = true;
  for_each_line(s, [&](const char *p, const char *end) {
    int x;
    if (!next_int(p, end, &x)) ok = false;
    d.split.push_back(ok ? x : 0);
  });
  return ok;
}

bool features_dense(const GCNData &d) {
  const int n = d.num_nodes, f = d.input_dim;
  if ((long long)d.feature_index.indptr.size() != (long long)n + 1) return false;
  for (int i = 0; i <= n; i++)
    if ((long long)d.feature_index.indptr[i] != (long long)i * f) return false;
  std::atomic<bool> dense{true};
  parallel_for((long long)n * f, [&](long long b, long long e) {
    for (long long j = b; j < e; j++)
      if (d.feature_index.indices[j] != (int)(j % f)) {
        dense = false;
        return;
      }
  });
  return dense;
}

// ------------------------------------------------------------------------------------------
// synthetic inputs
// ------------------------------------------------------------------------------------------
namespace {
inline uint64_t splitmix(uint64_t &x) {
  uint64_t z = (x += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
inline double u01(uint64_t &x) { return (double)(splitmix(x) >> 11) * 0x1.0p-53; }
inline uint64_t mix(uint64_t a, uint64_t b) {
  uint64_t x = a * 0x9e3779b97f4a7c15ull ^ (b + 0x632be59bd9b4e019ull);
  return splitmix(x);
}
}  // namespace

void make_synthetic(GCNData *d, int n, int f, int c, long long undirected_edges,
                    uint64_t seed) {
  // node weights: Pareto(alpha = 1.8), capped at 40x the mean
  std::vector<double> w((size_t)n);
  for (int i = 0; i < n; i++) {
    uint64_t st = mix(seed, 0x1000000000ull + (uint64_t)i);
    const double u = u01(st);
    w[(size_t)i] = std::pow(1.0 - u, -1.0 / 1.8);
  }
  double mean = 0;
  for (double x : w) mean += x;
  mean /= n;
  std::vector<double> cdf((size_t)n);
  double acc = 0;
  for (int i = 0; i < n; i++) {
    acc += std::min(w[(size_t)i], 40.0 * mean);
    cdf[(size_t)i] = acc;
  }
  auto sample = [&](uint64_t &st) {
    const double r = u01(st) * acc;
    int k = (int)(std::upper_bound(cdf.begin(), cdf.end(), r) - cdf.begin());
    return k >= n ? n - 1 : k;
  };
  // edges, generated in fixed blocks so the result does not depend on the thread count
  const long long M = undirected_edges;
  std::vector<int> eu((size_t)M), ev((size_t)M);
  const long long blk = 1 << 16;
  parallel_for(ceil_div(M, blk), [&](long long b0, long long b1) {
    for (long long b = b0; b < b1; b++) {
      uint64_t st = mix(seed, 0x2000000000ull + (uint64_t)b);
      for (long long e = b * blk; e < std::min(M, (b + 1) * blk); e++) {
        const int u = sample(st);
        int v = sample(st);
        while (v == u) v = sample(st);
        eu[(size_t)e] = u;
        ev[(size_t)e] = v;
      }
    }
  });
  // CSR: self loop first, then neighbours (both directions), sorted ascending
  std::vector<int> deg((size_t)n, 1);
  for (long long e = 0; e < M; e++) {
    deg[(size_t)eu[(size_t)e]]++;
    deg[(size_t)ev[(size_t)e]]++;
  }
  d->graph.indptr.assign((size_t)n + 1, 0);
  for (int i = 0; i < n; i++) d->graph.indptr[(size_t)i + 1] = d->graph.indptr[(size_t)i] + deg[(size_t)i];
  d->graph.indices.assign((size_t)d->graph.indptr[(size_t)n], 0);
  std::vector<int> fill(d->graph.indptr.begin(), d->graph.indptr.end() - 1);
  for (int i = 0; i < n; i++) d->graph.indices[(size_t)fill[(size_t)i]++] = i;
  for (long long e = 0; e < M; e++) {
    const int u = eu[(size_t)e], v = ev[(size_t)e];
    d->graph.indices[(size_t)fill[(size_t)u]++] = v;
    d->graph.indices[(size_t)fill[(size_t)v]++] = u;
  }
  std::vector<int>().swap(eu);
  std::vector<int>().swap(ev);
  parallel_for(n, [&](long long b, long long e) {
    for (long long i = b; i < e; i++)
      std::sort(d->graph.indices.begin() + d->graph.indptr[(size_t)i] + 1,
                d->graph.indices.begin() + d->graph.indptr[(size_t)i + 1]);
  });
  // dense features N(0,1) quantised to 4 decimals ("%.4f" in the text form), CSR layout
  d->feature_index.indptr.assign((size_t)n + 1, 0);
  for (int i = 0; i <= n; i++) d->feature_index.indptr[(size_t)i] = i * f;
  d->feature_index.indices.assign((size_t)n * f, 0);
  d->feature_value.assign((size_t)n * f, 0.0f);
  parallel_for(n, [&](long long b, long long e) {
    for (long long i = b; i < e; i++) {
      uint64_t st = mix(seed, 0x3000000000ull + (uint64_t)i);
      for (int k = 0; k < f; k += 2) {
        const double u1 = 1.0 - u01(st), u2 = u01(st);
        const double r = std::sqrt(-2.0 * std::log(u1));
        const double z[2] = {r * std::cos(2 * M_PI * u2), r * std::sin(2 * M_PI * u2)};
        for (int t = 0; t < 2 && k + t < f; t++) {
          const size_t idx = (size_t)i * f + k + t;
          d->feature_index.indices[idx] = k + t;
          d->feature_value[idx] = (float)(std::nearbyint(z[t] * 10000.0) / 10000.0);
        }
      }
    }
  });
  // labels uniform in [0, c); split by a seeded shuffle
  d->label.resize((size_t)n);
  for (int i = 0; i < n; i++) {
    uint64_t st = mix(seed, 0x4000000000ull + (uint64_t)i);
    d->label[(size_t)i] = (int)(splitmix(st) % (uint64_t)c);
  }
  std::vector<int> perm((size_t)n);
  for (int i = 0; i < n; i++) perm[(size_t)i] = i;
  uint64_t st = mix(seed, 0x5000000000ull);
  for (int i = n - 1; i > 0; i--) std::swap(perm[(size_t)i], perm[(size_t)(splitmix(st) % (uint64_t)(i + 1))]);
  const long long n_train = std::llround((double)n * 153431.0 / 232965.0);
  const long long n_val = std::llround((double)n * 23831.0 / 232965.0);
  d->split.assign((size_t)n, 3);
  for (long long k = 0; k < n; k++)
    d->split[(size_t)perm[(size_t)k]] = k < n_train ? 1 : (k < n_train + n_val ? 2 : 3);
  d->num_nodes = n;
  d->input_dim = f;
  d->output_dim = c;
}

// ------------------------------------------------------------------------------------------
// binary dataset cache
// ------------------------------------------------------------------------------------------
namespace {
constexpr char kMagic[8] = {'P', 'G', 'C', 'N', 'D', 'S', '0', '1'};

struct BinHeader {
  char magic[8];
  long long num_nodes, input_dim, output_dim, graph_nnz, feat_nnz;
  long long stamp[6];  // (size, mtime_ns) of .graph, .split, .svmlight
  unsigned long long checksum;
};

uint64_t fnv1a(uint64_t h, const void *p, size_t n) {
  const unsigned char *b = static_cast<const unsigned char *>(p);
  for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 1099511628211ull;
  return h;
}

template <class T>
uint64_t hash_vec(uint64_t h, const std::vector<T> &v) {
  return fnv1a(h, v.data(), v.size() * sizeof(T));
}

uint64_t payload_hash(const GCNData &d) {
  uint64_t h = 14695981039346656037ull;
  h = hash_vec(h, d.graph.indptr);
  h = hash_vec(h, d.graph.indices);
  h = hash_vec(h, d.feature_index.indptr);
  h = hash_vec(h, d.feature_index.indices);
  h = hash_vec(h, d.feature_value);
  h = hash_vec(h, d.label);
  h = hash_vec(h, d.split);
  return h;
}

template <class T>
bool write_vec(std::FILE *f, const std::vector<T> &v) {
  return v.empty() || std::fwrite(v.data(), sizeof(T), v.size(), f) == v.size();
}

template <class T>
bool read_vec(std::FILE *f, std::vector<T> &v, long long n) {
  if (n < 0) return false;
  v.resize((size_t)n);
  return n == 0 || std::fread(v.data(), sizeof(T), (size_t)n, f) == (size_t)n;
}
}  // namespace

bool stamp_file(const std::string &path, FileStamp *st) {
  struct stat sb;
  if (::stat(path.c_str(), &sb) != 0) return false;
  st->size = (long long)sb.st_size;
  st->mtime_ns = (long long)sb.st_mtim.tv_sec * 1000000000LL + (long long)sb.st_mtim.tv_nsec;
  return true;
}

bool save_binary(const GCNData &d, const std::string &path, const FileStamp stamps[3]) {
  BinHeader h{};
  std::memcpy(h.magic, kMagic, 8);
  h.num_nodes = d.num_nodes;
  h.input_dim = d.input_dim;
  h.output_dim = d.output_dim;
  h.graph_nnz = (long long)d.graph.indices.size();
  h.feat_nnz = (long long)d.feature_index.indices.size();
  for (int i = 0; i < 3; i++) {
    h.stamp[2 * i] = stamps ? stamps[i].size : -1;
    h.stamp[2 * i + 1] = stamps ? stamps[i].mtime_ns : -1;
  }
  h.checksum = payload_hash(d);
  const std::string tmp = path + ".tmp";
  std::FILE *f = std::fopen(tmp.c_str(), "wb");
  if (!f) return false;
  bool ok = std::fwrite(&h, sizeof(h), 1, f) == 1 && write_vec(f, d.graph.indptr) &&
            write_vec(f, d.graph.indices) && write_vec(f, d.feature_index.indptr) &&
            write_vec(f, d.feature_index.indices) && write_vec(f, d.feature_value) &&
            write_vec(f, d.label) && write_vec(f, d.split);
  ok = (std::fclose(f) == 0) && ok;
  if (ok) ok = std::rename(tmp.c_str(), path.c_str()) == 0;  // readers never see a partial file
  if (!ok) std::remove(tmp.c_str());
  return ok;
}

bool load_binary(GCNData *d, const std::string &path, const FileStamp *stamps) {
  std::FILE *f = std::fopen(path.c_str(), "rb");
  if (!f) return false;
  BinHeader h{};
  GCNData t;
  bool ok = std::fread(&h, sizeof(h), 1, f) == 1 && std::memcmp(h.magic, kMagic, 8) == 0 &&
            h.num_nodes >= 0 && h.num_nodes < INT_MAX;
  if (ok && stamps)
    for (int i = 0; i < 3; i++)
      ok = ok && h.stamp[2 * i] == stamps[i].size && h.stamp[2 * i + 1] == stamps[i].mtime_ns;
  const long long n = h.num_nodes;
  ok = ok && read_vec(f, t.graph.indptr, n + 1) && read_vec(f, t.graph.indices, h.graph_nnz) &&
       read_vec(f, t.feature_index.indptr, n + 1) &&
       read_vec(f, t.feature_index.indices, h.feat_nnz) &&
       read_vec(f, t.feature_value, h.feat_nnz) && read_vec(f, t.label, n) &&
       read_vec(f, t.split, n);
  ok = ok && std::fgetc(f) == EOF;  // nothing trailing
  std::fclose(f);
  ok = ok && t.graph.indptr.back() == h.graph_nnz && t.feature_index.indptr.back() == h.feat_nnz;
  if (!ok || payload_hash(t) != h.checksum) return false;
  t.num_nodes = (int)n;
  t.input_dim = (int)h.input_dim;
  t.output_dim = (int)h.output_dim;
  *d = std::move(t);
  return true;
}

bool load_dataset_cached(GCNData *d, const std::string &root, const std::string &name,
                         bool *from_cache) {
  const std::string base = root + "/data/" + name;
  FileStamp st[3];
  const bool stamped = stamp_file(base + ".graph", &st[0]) && stamp_file(base + ".split", &st[1]) &&
                       stamp_file(base + ".svmlight", &st[2]);
  const std::string cache = base + ".pgcnbin";
  if (from_cache) *from_cache = false;
  if (stamped && load_binary(d, cache, st)) {
    if (from_cache) *from_cache = true;
    return true;
  }
  Parser parser(d, name, root);
  if (!parser.parse()) return false;
  if (stamped) (void)save_binary(*d, cache, st);  // best effort (read-only data dirs)
  return true;
}

}  // namespace pgcn
