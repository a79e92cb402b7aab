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
#include <thread>

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

int g_parse_threads = 0;  // "parse_threads": host threads of Parser::parse (0 = up to 16)

namespace {

// Line-aligned pieces of buf for parallel parsing: piece k is [cut[k], cut[k+1]) and ends right
// after a '\n'; the text after the last '\n' belongs to no piece (the reference's getline/eof
// loop drops an unterminated last line, hpdga parser.cpp:23-27).
std::vector<size_t> line_pieces(const std::string &buf, int pieces) {
  const size_t last = buf.rfind('\n');
  const size_t end = last == std::string::npos ? 0 : last + 1;
  std::vector<size_t> cut(1, 0);
  for (int k = 1; k < pieces; k++) {
    size_t c = std::max(cut.back(), end * (size_t)k / (size_t)pieces);
    if (c > 0 && c < end && buf[c - 1] != '\n') {
      const size_t nl = buf.find('\n', c);
      c = nl == std::string::npos ? end : nl + 1;
    }
    cut.push_back(std::min(c, end));
  }
  cut.push_back(end);
  return cut;
}

int parse_threads(size_t bytes) {
  if (g_parse_threads > 0) return g_parse_threads;  // exactly this many pieces (tests)
  int t = (int)std::thread::hardware_concurrency();
  t = std::max(1, std::min(t, 16));  // the GPU box grants 16 CPUs per GPU
  // pieces of at least 1 MB (small files: one piece, no threads)
  return (int)std::max<size_t>(1, std::min<size_t>((size_t)t, bytes >> 20));
}

// Runs fn(piece, begin, end) for every '\n'-terminated line of each piece, pieces in
// parallel; fn sees the lines of one piece in file order.
template <class Fn>
void parallel_lines(const std::string &buf, const std::vector<size_t> &cut, Fn fn) {
  const int P = (int)cut.size() - 1;
  parallel_for(P, [&](long long p0, long long p1) {
    for (long long k = p0; k < p1; k++) {
      size_t pos = cut[(size_t)k];
      while (pos < cut[(size_t)k + 1]) {
        const size_t nl = buf.find('\n', pos);  // inside the piece: pieces end after a '\n'
        fn((int)k, buf.data() + pos, buf.data() + nl);
        pos = nl + 1;
      }
    }
  }, P, 2);
}

}  // namespace

bool Parser::parse() {
  std::string g, s, v;
  // isValidInput(): all three files must open (hpdga parser.cpp:50-53)
  if (!read_file(graph_path_, &g) || !read_file(split_path_, &s) || !read_file(svm_path_, &v))
    return false;
  GCNData &d = *data_;

  // parseGraph (hpdga parser.cpp:18-48).  Pieces parse in parallel; a line's implicit self
  // connection is its global line number, so each piece first learns how many lines precede it.
  {
    const std::vector<size_t> cut = line_pieces(g, parse_threads(g.size()));
    const int P = (int)cut.size() - 1;
    std::vector<long long> first((size_t)P + 1, 0);
    parallel_for(P, [&](long long p0, long long p1) {
      for (long long k = p0; k < p1; k++)
        first[(size_t)k + 1] = std::count(g.begin() + (long long)cut[(size_t)k],
                                          g.begin() + (long long)cut[(size_t)k + 1], '\n');
    }, P, 2);
    for (int k = 0; k < P; k++) first[(size_t)k + 1] += first[(size_t)k];
    PGCN_CHECK(first[(size_t)P] < INT_MAX, PGCN_E_INVALID, "parseGraph: too many lines");
    std::vector<std::vector<int>> len((size_t)P), idx((size_t)P);
    std::vector<int> line((size_t)P);
    for (int k = 0; k < P; k++) line[(size_t)k] = (int)first[(size_t)k];
    parallel_lines(g, cut, [&](int k, const char *p, const char *end) {
      std::vector<int> &ix = idx[(size_t)k];
      const size_t before = ix.size();
      ix.push_back(line[(size_t)k]++);  // implicit self connection
      int nb;
      while (next_int(p, end, &nb)) ix.push_back(nb);
      len[(size_t)k].push_back((int)(ix.size() - before));
    });
    const int n = (int)first[(size_t)P];
    d.graph.indptr.assign((size_t)n + 1, 0);
    std::vector<long long> base((size_t)P + 1, 0);
    for (int k = 0; k < P; k++) base[(size_t)k + 1] = base[(size_t)k] + (long long)idx[(size_t)k].size();
    PGCN_CHECK(base[(size_t)P] <= INT_MAX, PGCN_E_INVALID, "parseGraph: more than 2^31 slots");
    d.graph.indices.resize((size_t)base[(size_t)P]);
    parallel_for(P, [&](long long p0, long long p1) {
      for (long long k = p0; k < p1; k++) {
        std::copy(idx[(size_t)k].begin(), idx[(size_t)k].end(),
                  d.graph.indices.begin() + base[(size_t)k]);
        long long at = base[(size_t)k];
        for (size_t i = 0; i < len[(size_t)k].size(); i++) {
          at += len[(size_t)k][i];
          d.graph.indptr[(size_t)first[(size_t)k] + i + 1] = (int)at;
        }
      }
    }, P, 2);
    d.num_nodes = n;
  }

  // parseNode (hpdga parser.cpp:59-104), pieces in parallel, concatenated in file order
  {
    const std::vector<size_t> cut = line_pieces(v, parse_threads(v.size()));
    const int P = (int)cut.size() - 1;
    struct Piece {
      std::vector<int> len, label, idx;
      std::vector<float> val;
      int max_idx = 0, max_label = 0;
    };
    std::vector<Piece> pc((size_t)P);
    parallel_lines(v, cut, [&](int k, const char *p, const char *end) {
      Piece &o = pc[(size_t)k];
      const size_t before = o.idx.size();
      const char *q = p;
      while (q < end && is_ws(*q)) q++;
      if (q >= end) {  // nothing to extract: the sentry fails, label keeps its -1
        o.label.push_back(-1);
        o.len.push_back(0);
        return;
      }
      int label;
      if (!next_int(p, end, &label)) {  // a non-number: num_get stores 0 and fails
        o.label.push_back(0);
        o.len.push_back(0);
        return;
      }
      o.label.push_back(label);
      o.max_label = std::max(o.max_label, label);
      // "k:v" tokens
      while (true) {
        while (p < end && is_ws(*p)) p++;
        if (p >= end) break;
        const char *tok = p;
        while (p < end && !is_ws(*p)) p++;
        const char *tend = p;
        int kk = 0;
        const char *t = tok;
        next_int(t, tend, &kk);
        if (t < tend) t++;  // the ':' (kv_ss >> col)
        char num[64];
        size_t nn = std::min((size_t)(tend - t), sizeof num - 1);
        std::memcpy(num, t, nn);
        num[nn] = 0;
        o.val.push_back(std::strtof(num, nullptr));
        o.idx.push_back(kk);
        o.max_idx = std::max(o.max_idx, kk);
      }
      o.len.push_back((int)(o.idx.size() - before));
    });
    long long rows = 0, nnz = 0;
    std::vector<long long> row0((size_t)P + 1, 0), nz0((size_t)P + 1, 0);
    int max_idx = 0, max_label = 0;
    for (int k = 0; k < P; k++) {
      row0[(size_t)k + 1] = rows += (long long)pc[(size_t)k].label.size();
      nz0[(size_t)k + 1] = nnz += (long long)pc[(size_t)k].idx.size();
      max_idx = std::max(max_idx, pc[(size_t)k].max_idx);
      max_label = std::max(max_label, pc[(size_t)k].max_label);
    }
    PGCN_CHECK(nnz <= INT_MAX, PGCN_E_INVALID, "parseNode: more than 2^31 features");
    d.feature_index.indptr.assign((size_t)rows + 1, 0);
    d.feature_index.indices.resize((size_t)nnz);
    d.feature_value.resize((size_t)nnz);
    d.label.resize((size_t)rows);
    parallel_for(P, [&](long long p0, long long p1) {
      for (long long k = p0; k < p1; k++) {
        const Piece &o = pc[(size_t)k];
        std::copy(o.idx.begin(), o.idx.end(), d.feature_index.indices.begin() + nz0[(size_t)k]);
        std::copy(o.val.begin(), o.val.end(), d.feature_value.begin() + nz0[(size_t)k]);
        std::copy(o.label.begin(), o.label.end(), d.label.begin() + row0[(size_t)k]);
        long long at = nz0[(size_t)k];
        for (size_t i = 0; i < o.len.size(); i++) {
          at += o.len[i];
          d.feature_index.indptr[(size_t)row0[(size_t)k] + i + 1] = (int)at;
        }
      }
    }, P, 2);
    d.input_dim = max_idx + 1;
    d.output_dim = max_label + 1;
  }

  // parseSplit (hpdga parser.cpp:106-116): std::stoi per line (small: one pass)
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
