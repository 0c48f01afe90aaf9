// dataset.h -- interaction data (reference: dataset.h:25-99).
//
// Dataset(filename) parses a `uid,sid` CSV.  The header line is always
// skipped (the reference skips it inside an assert, dataset.h:80, which its
// build keeps live -- SURVEY App. A.3).  Each entity's history keeps FILE
// ORDER (dataset.h:87-88), which the ProjectV tail quirk depends on.
//
// Storage is CSR per orientation (int64 row_ptr, int32 col), the layout the
// device consumes; the reference's unordered_map<int, SpVector> views
// (by_user()/by_item()) are built on first use for API compatibility.
#pragma once

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <thread>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "frecsys/logging.h"
#include "frecsys/types.h"

namespace frecsys {

struct Csr {
  std::vector<int64_t> ptr;  // rows + 1
  std::vector<int32_t> col;  // other-side ids, file order within a row
  int64_t rows() const { return ptr.empty() ? 0 : (int64_t)ptr.size() - 1; }
  int64_t len(int64_t r) const { return ptr[r + 1] - ptr[r]; }
};

namespace detail {
// Counting sort of (row, col) pairs by row, stable: keeps file order.
inline Csr build_csr(const std::vector<int32_t>& rows, const std::vector<int32_t>& cols,
                     int64_t n_rows) {
  Csr c;
  c.ptr.assign((size_t)n_rows + 1, 0);
  for (int32_t r : rows) c.ptr[(size_t)r + 1]++;
  for (int64_t i = 0; i < n_rows; ++i) c.ptr[i + 1] += c.ptr[i];
  c.col.resize(rows.size());
  std::vector<int64_t> fill(c.ptr.begin(), c.ptr.end() - 1);
  for (size_t k = 0; k < rows.size(); ++k) c.col[(size_t)fill[rows[k]]++] = cols[k];
  return c;
}
// Rating index (tuple position) of every entry of build_csr(rows, ...):
// the same stable counting sort, storing positions.
inline std::vector<int32_t> build_rix(const std::vector<int32_t>& rows, int64_t n_rows) {
  std::vector<int64_t> fill((size_t)n_rows + 1, 0);
  for (int32_t r : rows) fill[(size_t)r + 1]++;
  for (int64_t i = 0; i < n_rows; ++i) fill[i + 1] += fill[i];
  std::vector<int32_t> rix(rows.size());
  for (size_t k = 0; k < rows.size(); ++k) rix[(size_t)fill[rows[k]]++] = (int32_t)k;
  return rix;
}
}  // namespace detail

class Dataset {
 public:
  explicit Dataset(const std::string& filename) {
    int fd = open(filename.c_str(), O_RDONLY);
    if (fd < 0) throw std::runtime_error("cannot open " + filename);
    struct stat st;
    fstat(fd, &st);
    size_t n = (size_t)st.st_size;
    const char* p = n ? (const char*)mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0) : nullptr;
    const char* end = p + n;
    const char* q = p;
    while (q < end && *q != '\n') ++q;  // discard header (dataset.h:79-80)
    if (q < end) ++q;
    // Parallel parse: the body is cut into chunks at
    // line boundaries, parsed by one thread each, and concatenated in chunk
    // order -- the tuples keep file order exactly as a sequential read.
    const size_t body = (size_t)(end - q);
    int nt = (int)std::min<size_t>(std::max(1u, std::thread::hardware_concurrency()), 16);
    if (const char* e = getenv("FRECSYS_LOAD_THREADS")) nt = std::max(1, atoi(e));
    if (body < ((size_t)1 << 20)) nt = 1;
    std::vector<const char*> cut((size_t)nt + 1, end);
    cut[0] = q;
    for (int t = 1; t < nt; ++t) {
      const char* c = q + body * t / nt;
      if (c < cut[t - 1]) c = cut[t - 1];
      while (c < end && c[-1] != '\n') ++c;  // start of the next line
      cut[t] = c;
    }
    std::vector<std::vector<int32_t>> us((size_t)nt), is((size_t)nt);
    auto parse = [&](int t) { parse_lines(cut[t], cut[t + 1], &us[t], &is[t]); };
    if (nt == 1) {
      parse(0);
    } else {
      std::vector<std::thread> th;
      for (int t = 0; t < nt; ++t) th.emplace_back(parse, t);
      for (auto& x : th) x.join();
    }
    size_t total = 0;
    for (int t = 0; t < nt; ++t) total += us[t].size();
    users_.reserve(total);
    items_.reserve(total);
    for (int t = 0; t < nt; ++t) {
      users_.insert(users_.end(), us[t].begin(), us[t].end());
      items_.insert(items_.end(), is[t].begin(), is[t].end());
    }
    if (p) munmap((void*)p, n);
    close(fd);
    finish();
  }

  // Programmatic construction (synthetic data, tests); rows in the given
  // ("file") order.
  Dataset(std::vector<int32_t> users, std::vector<int32_t> items)
      : users_(std::move(users)), items_(std::move(items)) {
    finish();
  }

  int max_user() const { return max_user_; }
  int max_item() const { return max_item_; }
  int num_tuples() const { return (int)users_.size(); }
  const std::vector<int32_t>& users() const { return users_; }
  const std::vector<int32_t>& items() const { return items_; }

  // CSR views sized max_user+1 / max_item+1 (rows with no history are empty).
  const Csr& user_csr() const {
    std::call_once(csr_once_[0], [&] { ucsr_ = detail::build_csr(users_, items_, max_user_ + 1); });
    return ucsr_;
  }
  const Csr& item_csr() const {
    std::call_once(csr_once_[1], [&] { icsr_ = detail::build_csr(items_, users_, max_item_ + 1); });
    return icsr_;
  }

  // Rating index of every CSR entry (the second member of the reference's
  // by_user / by_item pairs), in CSR order.
  std::vector<int32_t> user_rix() const { return detail::build_rix(users_, max_user_ + 1); }
  std::vector<int32_t> item_rix() const { return detail::build_rix(items_, max_item_ + 1); }

  // Reference API: SpMatrix with (other id, rating index) pairs.
  const SpMatrix& by_user() const {
    std::call_once(map_once_[0], [&] {
      for (size_t k = 0; k < users_.size(); ++k) by_user_[users_[k]].push_back({items_[k], (int)k});
    });
    return by_user_;
  }
  const SpMatrix& by_item() const {
    std::call_once(map_once_[1], [&] {
      for (size_t k = 0; k < users_.size(); ++k) by_item_[items_[k]].push_back({users_[k], (int)k});
    });
    return by_item_;
  }

  // Distinct users, ascending, and their compacted CSR (the fold-in's
  // user_to_ind, ials.h:151-166).
  void compact_users(std::vector<int32_t>* ids, Csr* csr) const {
    const Csr& u = user_csr();
    ids->clear();
    csr->ptr.assign(1, 0);
    csr->col.clear();
    for (int64_t r = 0; r < u.rows(); ++r) {
      if (u.len(r) == 0) continue;
      ids->push_back((int32_t)r);
      csr->col.insert(csr->col.end(), u.col.begin() + u.ptr[r], u.col.begin() + u.ptr[r + 1]);
      csr->ptr.push_back((int64_t)csr->col.size());
    }
  }

  // merge() of the reference is a no-op (it copies the target by value,
  // dataset.h:43-61) and unused; it is deliberately not provided.

 private:
  // "user,item" lines of [q, end); atoi semantics (dataset.h:84-85).
  static void parse_lines(const char* q, const char* end, std::vector<int32_t>* users,
                          std::vector<int32_t>* items) {
    while (q < end) {
      const char* ls = q;
      while (q < end && *q != '\n') ++q;
      const char* le = q;
      if (q < end) ++q;
      if (le > ls && le[-1] == '\r') --le;
      if (le == ls) continue;
      const char* comma = ls;
      while (comma < le && *comma != ',') ++comma;
      users->push_back(parse_int(ls, comma));
      items->push_back(comma < le ? parse_int(comma + 1, le) : 0);
    }
  }
  static int32_t parse_int(const char* b, const char* e) {
    while (b < e && (*b == ' ' || *b == '\t')) ++b;
    bool neg = false;
    if (b < e && (*b == '-' || *b == '+')) neg = *b++ == '-';
    int64_t v = 0;
    while (b < e && *b >= '0' && *b <= '9') v = v * 10 + (*b++ - '0');
    return (int32_t)(neg ? -v : v);
  }
  void finish() {
    max_user_ = -1;
    max_item_ = -1;
    for (size_t k = 0; k < users_.size(); ++k) {
      max_user_ = std::max(max_user_, (int)users_[k]);
      max_item_ = std::max(max_item_, (int)items_[k]);
    }
    int64_t du = 0, di = 0;
    {
      std::vector<char> su((size_t)max_user_ + 1, 0), si((size_t)max_item_ + 1, 0);
      for (size_t k = 0; k < users_.size(); ++k) {
        du += !su[users_[k]];
        su[users_[k]] = 1;
        di += !si[items_[k]];
        si[items_[k]] = 1;
      }
    }
    LOG(INFO) << "max_user=" << max_user_ << "\tmax_item=" << max_item_
              << "\tdistinct user=" << du << "\tdistinct item=" << di
              << "\tnum_tuples=" << num_tuples();  // dataset.h:94-98
  }

  std::vector<int32_t> users_, items_;
  int max_user_ = -1, max_item_ = -1;
  mutable std::once_flag csr_once_[2], map_once_[2];
  mutable Csr ucsr_, icsr_;
  mutable SpMatrix by_user_, by_item_;
};

}  // namespace frecsys
