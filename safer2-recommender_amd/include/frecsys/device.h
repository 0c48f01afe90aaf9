// device.h -- C++ side of the drop-in boundary: a RAII owner of one
// frecsys_ctx (include/frecsys_hip.h) used by the model classes.
//
// It keeps the training data resident (both CSR orientations), tracks which
// Gramian each slot holds so an unchanged G is not recomputed (the
// reference recomputes V^T V in every Step, ials.h:321/371 -- same values,
// the kernels are deterministic), and turns C-ABI status codes into the
// reference's visible behaviour: a failed LLT is an assert in the reference
// (ials.h:141) -> LOG(FATAL) (abort) here, naming the entity.
#pragma once

#include <array>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "frecsys/dataset.h"
#include "frecsys/logging.h"
#include "frecsys/types.h"
#include "frecsys_hip.h"

namespace frecsys {

// Optional tail of every model ctor (the reference signatures are kept).
struct DeviceOptions {
  int64_t seed = -1;          // -1: std::random_device, as the reference (ials.h:48)
  int device = -1;            // HIP ordinal; -1: LOCAL_RANK or the current device
  bool parity_quirks = true;  // SURVEY App. A.1 (ProjectV tail double count)
  int world = 0;              // 0: from WORLD_SIZE (1 if unset)
  int rank = -1;              // -1: from RANK
  std::string comm_file;      // RCCL id rendezvous file for world > 1
  bool has_comm_id = false;   // comm_id given by the caller (e.g. exchanged over
  std::array<uint8_t, 128> comm_id{};  // torch.distributed): no file rendezvous

  static DeviceOptions FromEnv() {
    DeviceOptions o;
    if (const char* s = getenv("FRECSYS_SEED")) o.seed = atoll(s);
    return o;
  }
};

inline int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return v && *v ? atoi(v) : dflt;
}

class DeviceContext {
 public:
  enum Side { USER = FRECSYS_SIDE_USER, ITEM = FRECSYS_SIDE_ITEM, EVAL = FRECSYS_SIDE_EVAL };

  DeviceContext(int dim, int64_t n_users, int64_t n_items, const DeviceOptions& o)
      : dim_(dim), n_{n_users, n_items, 0} {
    world_ = o.world > 0 ? o.world : env_int("WORLD_SIZE", 1);
    rank_ = o.rank >= 0 ? o.rank : env_int("RANK", 0);
    frecsys_config cfg;
    std::memset(&cfg, 0, sizeof(cfg));
    cfg.dim = dim;
    cfg.device = o.device >= 0 ? o.device : (world_ > 1 ? env_int("LOCAL_RANK", 0) : -1);
    cfg.parity_quirks = o.parity_quirks ? 1 : 0;
    cfg.n_users = n_users;
    cfg.n_items = n_items;
    check(frecsys_ctx_create(&cfg, &ctx_), "frecsys_ctx_create");
    if (world_ > 1) comm_init(o);
  }
  ~DeviceContext() {
    if (ctx_) frecsys_ctx_destroy(ctx_);
  }
  DeviceContext(const DeviceContext&) = delete;
  DeviceContext& operator=(const DeviceContext&) = delete;

  frecsys_ctx* raw() { return ctx_; }
  int dim() const { return dim_; }
  int world() const { return world_; }
  int rank() const { return rank_; }
  int64_t rows(int side) const { return n_[side]; }

  // ---- data ----
  void LoadTraining(const Dataset& d) {
    if (loaded_ == &d && loaded_tuples_ == d.num_tuples()) return;
    const Csr& u = d.user_csr();
    const Csr& i = d.item_csr();
    load_side(USER, u, n_[USER]);
    load_side(ITEM, i, n_[ITEM]);
    loaded_ = &d;
    loaded_tuples_ = d.num_tuples();
  }
  void LoadEval(const Csr& c) {
    check(frecsys_load_csr(ctx_, EVAL, c.rows(), c.ptr.data(), c.col.data()), "load_csr(eval)");
    n_[EVAL] = c.rows();
  }

  // ---- embeddings ----
  void InitEmbeddings(int64_t seed, float stdev) {
    uint32_t s = seed >= 0 ? (uint32_t)seed : (uint32_t)std::random_device{}();
    check(frecsys_init_embeddings(ctx_, s, stdev), "init_embeddings");
    bump(USER);
    bump(ITEM);
  }
  MatrixXf Get(int side) {
    MatrixXf m(n_[side], dim_);
    check(frecsys_get_embeddings(ctx_, side, m.data(), dim_), "get_embeddings");
    return m;
  }
  void Set(int side, const MatrixXf& m) {
    check(frecsys_set_embeddings(ctx_, side, m.data(), dim_), "set_embeddings");
    bump(side);
  }
  void Snapshot(int side) { check(frecsys_snapshot(ctx_, side), "snapshot"); }
  // ||X - snapshot|| over every row of side (the residual norms of
  // --print_residual_stats), on the device; sqrt of a double sum.
  float SnapshotResidual(int side) {
    double sq = 0.0;
    check(frecsys_snapshot_residual(ctx_, side, &sq), "snapshot_residual");
    return (float)std::sqrt(sq);
  }

  // ---- Gramians: slot `side` holds G of side's embeddings, optionally
  //      weighted; recomputed only when the embeddings or weights changed.
  void Gramian(int side, const float* weights = nullptr, uint64_t weight_tag = 0,
               bool from_snapshot = false) {
    const uint64_t key = (version_[side] << 1) ^ (weights ? (weight_tag * 0x9E3779B97F4A7C15ull | 1) : 0);
    if (!from_snapshot && gram_key_[side] == key && gram_valid_[side]) return;
    check(frecsys_gramian(ctx_, side, weights, from_snapshot ? 1 : 0, nullptr), "gramian");
    gram_key_[side] = key;
    gram_valid_[side] = !from_snapshot;
  }
  void InvalidateGramian(int side) { gram_valid_[side] = false; }

  // ---- the per-entity solve loop of one side ----
  void Solve(int side, const frecsys_solve_params& p) {
    int rc = frecsys_solve_side(ctx_, side, &p);
    if (rc == FRECSYS_ERR_NOT_SPD) {
      // reference: assert(cholesky.info() == Eigen::Success), ials.h:141
      LOG(FATAL) << "LLT failed: normal-equation matrix not SPD for entity "
                 << frecsys_last_error_entity(ctx_) << " (side " << side << ")";
    }
    check(rc, "solve_side");
    if (side != EVAL) bump(side);
  }

  // ---- iALS++ (ialspp.h) ----
  void PPLoad(const Dataset& d) {
    LoadTraining(d);
    if (pp_loaded_ == &d && pp_tuples_ == d.num_tuples()) return;
    const std::vector<int32_t> ur = d.user_rix(), ir = d.item_rix();
    check(frecsys_pp_set_rating_index(ctx_, USER, ur.data()), "pp_set_rating_index(user)");
    check(frecsys_pp_set_rating_index(ctx_, ITEM, ir.data()), "pp_set_rating_index(item)");
    pp_loaded_ = &d;
    pp_tuples_ = d.num_tuples();
  }
  void PPPredict(int side) { check(frecsys_pp_predict(ctx_, side), "pp_predict"); }
  double PPStep(int side, int start, int end, const frecsys_solve_params& p) {
    double r = 0.0;
    const int rc = frecsys_pp_step(ctx_, side, start, end, &p, &r);
    if (rc == FRECSYS_ERR_NOT_SPD)
      LOG(FATAL) << "LLT failed in ProjectBlock for entity " << frecsys_last_error_entity(ctx_);
    check(rc, "pp_step");
    if (side != EVAL) bump(side);
    return r;
  }
  // Zero the EVAL embeddings (the fold-in starts from 0, ialspp.h:155-170).
  void ZeroEval(int dim) {
    std::vector<float> z((size_t)n_[EVAL] * dim, 0.0f);
    if (n_[EVAL]) check(frecsys_set_embeddings(ctx_, EVAL, z.data(), dim), "set_embeddings(eval)");
  }

  // ComputeLosses parts on the GPU (frecsys_train_stats).
  void TrainStats(double* observed, double* unobserved, float* user_norm2, float* item_norm2) {
    check(frecsys_train_stats(ctx_, observed, unobserved, user_norm2, item_norm2), "train_stats");
  }

  // Best k items per EVAL row (history excluded), [rows][k] (GPU scoring + top-k).
  std::vector<int32_t> EvalTopK(int k) {
    std::vector<int32_t> out((size_t)n_[EVAL] * k);
    check(frecsys_eval_topk(ctx_, k, out.data()), "eval_topk");
    return out;
  }

  // Per-user loss of `side` (USER or EVAL) against ITEM / G[ITEM].
  void UserLoss(int side, float beta, bool half, float* host_out) {
    check(frecsys_user_loss(ctx_, side, beta, half ? 1 : 0, host_out), "user_loss");
  }

  void check(int rc, const char* what) {
    if (rc != FRECSYS_OK)
      LOG(FATAL) << what << " failed (" << rc << "): " << frecsys_last_error(ctx_);
  }

 private:
  void bump(int side) {
    if (side < 2) {
      ++version_[side];
      gram_valid_[side] = false;
    }
  }
  void load_side(int side, const Csr& c, int64_t rows) {
    // the model is sized from the training set (run_model.cc:239-240); a
    // CSR with fewer rows is padded with empty rows
    std::vector<int64_t> ptr(c.ptr);
    if ((int64_t)ptr.size() < rows + 1) ptr.resize((size_t)rows + 1, ptr.empty() ? 0 : ptr.back());
    check(frecsys_load_csr(ctx_, side, rows, ptr.data(), c.col.data()), "load_csr");
  }
  void comm_init(const DeviceOptions& o) {
    if (o.has_comm_id) {
      check(frecsys_comm_init(ctx_, world_, rank_, o.comm_id.data()), "comm_init");
      return;
    }
    std::string path = o.comm_file;
    if (path.empty()) {
      const char* f = getenv("FRECSYS_COMM_FILE");
      path = f ? f : "/tmp/frecsys_rccl_" + std::string(getenv("MASTER_PORT") ? getenv("MASTER_PORT") : "0");
    }
    uint8_t id[128];
    if (rank_ == 0) {
      check(frecsys_comm_unique_id(id), "comm_unique_id");
      std::string tmp = path + ".tmp";
      std::ofstream(tmp, std::ios::binary).write((const char*)id, 128);
      std::rename(tmp.c_str(), path.c_str());
    } else {
      for (int tries = 0;; ++tries) {
        std::ifstream f(path, std::ios::binary);
        if (f && f.read((char*)id, 128) && f.gcount() == 128) break;
        if (tries > 6000) LOG(FATAL) << "no RCCL id at " << path;
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
      }
    }
    check(frecsys_comm_init(ctx_, world_, rank_, id), "comm_init");
  }

  frecsys_ctx* ctx_ = nullptr;
  int dim_;
  int64_t n_[3];
  int world_ = 1, rank_ = 0;
  const Dataset* loaded_ = nullptr;
  int loaded_tuples_ = -1;
  uint64_t version_[2] = {1, 1};
  const Dataset* pp_loaded_ = nullptr;
  int pp_tuples_ = -1;
  uint64_t gram_key_[2] = {0, 0};
  bool gram_valid_[2] = {false, false};
};

inline frecsys_solve_params solve_params(int kind, float reg, float w) {
  frecsys_solve_params p;
  std::memset(&p, 0, sizeof(p));
  p.kind = kind;
  p.reg = reg;
  p.reg_exp = 1.0f;
  p.unobserved_weight = w;
  return p;
}

}  // namespace frecsys
