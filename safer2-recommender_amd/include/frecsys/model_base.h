// model_base.h -- state and helpers shared by the four GPU model classes.
//
// Host-resident: the small per-user vectors of the reference models
// (user_loss_, dual_weight_, user_history_size_, item_reg_; safer2.h:841-847)
// and the print flags.  Device-resident (DeviceContext): U, V, Gramians,
// the CSR of the training set.  The static per-entity entry points
// (Project / ProjectU / ProjectV of the reference) run on the GPU through a
// one-row context (ProjectOnDevice).
#pragma once

#include <chrono>
#include <cmath>
#include <cstring>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "frecsys/dataset.h"
#include "frecsys/device.h"
#include "frecsys/evaluation.h"
#include "frecsys/logging.h"
#include "frecsys/recommender.h"
#include "frecsys/types.h"

namespace frecsys {
namespace detail {

class DeviceModel : public Recommender {
 public:
  DeviceModel(int dim, int num_users, int num_items, float stdev, const DeviceOptions& opts)
      : dim_(dim), num_users_(num_users), num_items_(num_items), opts_(opts) {
    dev_ = std::make_unique<DeviceContext>(dim, num_users, num_items, opts);
    // adjusted_stdev = stdev / sqrt(dim); U then V from one mt19937
    // (ials.h:47-51 / recommender.h:61-67)
    dev_->InitEmbeddings(opts.seed, stdev);
  }

  void SetPrintTrainStats(const bool v) override { print_trainstats_ = v; }
  void SetPrintResidualStats(const bool v) override { print_residualstats_ = v; }
  void SetPrintVarStats(const bool v) override { print_varstats_ = v; }

  // Host copies of the device embeddings (item_embedding(), ials.h:410).
  MatrixXf item_embedding() const { return dev_->Get(DeviceContext::ITEM); }
  MatrixXf user_embedding() const { return dev_->Get(DeviceContext::USER); }
  void set_embeddings(const MatrixXf& U, const MatrixXf& V) {
    dev_->Set(DeviceContext::USER, U);
    dev_->Set(DeviceContext::ITEM, V);
    OnEmbeddingsSet();
  }
  const VectorXf& user_loss() const { return user_loss_; }
  // The dual state of ERM-MF / CVaR-MF / SAFER2 (empty for iALS): omega as
  // the last Train() used it, and item_reg_ from Initialize().
  const VectorXf& dual_weights() const { return dual_weight_; }
  const VectorXf& item_regularization() const { return item_reg_; }
  DeviceContext& device() { return *dev_; }

 protected:
  virtual void OnEmbeddingsSet() {}

  // Fold-in + evaluation (ials.h:148-185 and its model variants, then
  // EvaluateDatasetInternal / EvaluateUser, recommender.h:78-199): project
  // the users of `data` with `params`, score every item, exclude each user's
  // fold-in history and rank -- all on the GPU (frecsys_eval_topk); Recall /
  // NDCG of the k_list cut-offs on host.
  EvaluationResult FoldInEvaluate(const VectorXi& k_list, const VectorXf& alpha_list,
                                  const Dataset& data, const SpMatrix& eval_by_user,
                                  const frecsys_solve_params& params) {
    std::vector<int32_t> ids;
    Csr csr;
    data.compact_users(&ids, &csr);
    dev_->LoadEval(csr);
    dev_->Solve(DeviceContext::EVAL, params);
    return RankEval(k_list, alpha_list, ids, eval_by_user);
  }

  // Ranking of the projected EVAL rows (ids = their user ids): GPU scoring +
  // top-K, Recall / NDCG on host (recommender.h:132-199).
  EvaluationResult RankEval(const VectorXi& k_list, const VectorXf& alpha_list,
                            const std::vector<int32_t>& ids, const SpMatrix& eval_by_user) {
    const int max_k = std::min<int>(k_list.maxCoeff(), (int)num_items_);
    const std::vector<int32_t> top = dev_->EvalTopK(max_k);
    std::unordered_map<int, int> user_to_ind;
    for (size_t i = 0; i < ids.size(); ++i) user_to_ind[ids[i]] = (int)i;
    const int64_t nk = k_list.size();
    const int64_t nu = (int64_t)eval_by_user.size();
    MatrixXf recall = MatrixXf::Zero(nu, nk), ndcg = MatrixXf::Zero(nu, nk);
    int row = 0;
    for (const auto& kv : eval_by_user) {
      const int32_t* t = top.data() + (size_t)user_to_ind.at(kv.first) * max_k;
      const UserEvaluationResult m = RankMetrics(k_list, t, max_k, kv.second);
      for (int64_t i = 0; i < nk; ++i) {
        recall(row, i) = m.recall[i];
        ndcg(row, i) = m.ndcg[i];
      }
      ++row;
    }
    return EvaluationResult{k_list, alpha_list, recall, ndcg};
  }

  // Initialize() bookkeeping of ERM-MF / CVaR-MF / SAFER2
  // (safer2.h:827-837): |H_u| and item_reg_[v] = sum_{u in H_v} 1/|H_u|
  // accumulated in by_item (file) order.
  void ComputeHistoryStats(const Dataset& data) {
    user_history_size_ = VectorXf::Zero(num_users_);
    item_reg_ = VectorXf::Zero(num_items_);
    const Csr& u = data.user_csr();
    const Csr& it = data.item_csr();
    for (int64_t r = 0; r < u.rows() && r < num_users_; ++r) user_history_size_[r] = (float)u.len(r);
    for (int64_t v = 0; v < it.rows() && v < num_items_; ++v)
      for (int64_t k = it.ptr[v]; k < it.ptr[v + 1]; ++k)
        item_reg_[v] = (float)((double)item_reg_[v] + 1.0 / (double)user_history_size_[it.col[k]]);
  }

  // VaR / CVaR of the user losses (safer2.h:304-316).
  void PrintVarStats(float alpha) const {
    std::vector<float> vals((size_t)user_loss_.size());
    for (int64_t i = 0; i < user_loss_.size(); ++i) vals[i] = -user_loss_[i];
    const size_t Q = (size_t)((float)vals.size() * alpha);
    std::nth_element(vals.begin(), vals.begin() + Q, vals.end());
    float loss = 0;
    for (size_t i = 0; i <= Q; i++) loss += -vals[i];
    LOG(INFO) << "VaR: " << -vals[Q] << " CVaR: " << loss / (float)Q;
  }

  // Train-loss diagnostics (ials.h:226-305, safer2.h:337-413): the
  // observed / unobserved sums and the squared row norms of U and V, computed
  // on the GPU (frecsys_train_stats); counted in Train() time like the
  // reference's (run_model flag --print_train_stats, default on).
  struct LossParts {
    double observed = 0, unobserved = 0;
    std::vector<float> user_norm2, item_norm2;
  };
  LossParts ComputeLossParts(const Dataset& data) {
    (void)data;
    LossParts lp;
    lp.user_norm2.resize((size_t)num_users_);
    lp.item_norm2.resize((size_t)num_items_);
    dev_->TrainStats(&lp.observed, &lp.unobserved, lp.user_norm2.data(), lp.item_norm2.data());
    return lp;
  }

  // PrintLosses of the weighted models (safer2.h:337-413, erm_mf.h:303-377,
  // cvar_mf.h:332-406 -- identical): loss = sum of the user losses, the
  // regularisers with UserRegularizationValue / ItemRegularizationValue.
  void PrintWeightedLosses(const Dataset& data, float reg, float w, float alpha) {
    if (!print_trainstats_) return;
    const auto t0 = std::chrono::steady_clock::now();
    const LossParts lp = ComputeLossParts(data);
    const Csr& uc = data.user_csr();
    const Csr& ic = data.item_csr();
    float loss_reg = 0.0f, reg_user_now = 0.0f, reg_item_now = 0.0f;
    for (int64_t u = 0; u < uc.rows(); ++u) {
      if (!uc.len(u)) continue;
      const float n2 = lp.user_norm2[u];
      loss_reg += n2 * (reg * (1 + w * num_items_));
      reg_user_now += n2;
    }
    for (int64_t i = 0; i < ic.rows(); ++i) {
      if (!ic.len(i)) continue;
      const float n2 = lp.item_norm2[i];
      loss_reg += n2 * (reg * (item_reg_[i] + alpha * w * num_users_));
      reg_item_now += n2;
    }
    const float loss = user_loss_.sum();
    const auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(
                        std::chrono::steady_clock::now() - t0)
                        .count();
    CheckNaN(loss);
    LOG(INFO) << format(
        "Loss={0:.2f} Loss_observed={1:.2f} Loss_unobserved={2:.2f} Loss_reg={3:.2f} "
        "Loss_reg (user)={4:.2f} Loss_reg (item)={5:.2f}",
        loss, lp.observed / data.num_tuples(), lp.unobserved / num_items_ / num_users_, loss_reg,
        reg_user_now / num_users_, reg_item_now / num_items_);
    LOG(INFO) << format("Time={0}", (int64_t)ms);
  }

  // (w - w_prev).norm() of the dual weights (ComputeUserWeights' residual,
  // safer2.h:789-792, cvar_mf.h:637-640), in double.
  static float WeightResidual(const VectorXf& w, const VectorXf& prev) {
    double s = 0.0;
    for (int64_t i = 0; i < w.size(); ++i) {
      const double d = (double)w[i] - (double)prev[i];
      s += d * d;
    }
    return (float)std::sqrt(s);
  }

  static double RowSqNorm(const MatrixXf& M, int64_t r) {
    double s = 0;
    for (int64_t j = 0; j < M.cols(); ++j) s += (double)M(r, j) * M(r, j);
    return s;
  }

  void CheckNaN(float loss) const {
    if (std::isnan(loss)) {  // ials.h:291-296: logged, then exit(0)
      LOG(ERROR) << "!!!!!!!!!!!!!!!!!!!!!!!!!!!!!!!!!!!!!";
      LOG(ERROR) << "NaN is detected!!";
      LOG(ERROR) << "!!!!!!!!!!!!!!!!!!!!!!!!!!!!!!!!!!!!!";
      std::exit(0);
    }
  }

  int dim_;
  int64_t num_users_, num_items_;
  DeviceOptions opts_;
  std::unique_ptr<DeviceContext> dev_;
  VectorXf user_loss_;
  VectorXf dual_weight_;
  VectorXf user_history_size_;
  VectorXf item_reg_;
  bool print_trainstats_ = false;
  bool print_residualstats_ = false;  // uninitialised in the reference
  bool print_varstats_ = false;
};

inline void check_ok(int rc) {
  if (rc != FRECSYS_OK) LOG(FATAL) << "frecsys call failed (" << rc << "): " << frecsys_last_error(nullptr);
}

// One-entity projection through a temporary device context: the reference's
// static Project / ProjectU / ProjectV (ials.h:88, safer2.h:104, 166) with
// `reg` used as the final lambda.
inline VectorXf ProjectOnDevice(int kind, const SpVector& history, const MatrixXf& X,
                                const MatrixXf& G, float reg, float w, float weight,
                                const VectorXf* nu) {
  const int d = (int)X.cols();
  DeviceOptions o;
  o.world = 1;
  o.rank = 0;
  DeviceContext ctx(d, 1, X.rows(), o);
  Csr c;
  c.ptr = {0, (int64_t)history.size()};
  for (const auto& p : history) c.col.push_back(p.first);
  // side USER (1 row) against ITEM = X
  check_ok(frecsys_load_csr(ctx.raw(), FRECSYS_SIDE_USER, 1, c.ptr.data(), c.col.data()));
  ctx.Set(DeviceContext::ITEM, X);
  check_ok(frecsys_set_gramian(ctx.raw(), FRECSYS_SIDE_ITEM, G.data(), d));
  frecsys_solve_params p = solve_params(kind, reg, w);
  p.lambda_is_reg = 1;
  float om = weight;
  std::vector<float> er(1, 0.0f);
  std::vector<float> nuv;
  if (kind == FRECSYS_KIND_WEIGHTED_U) p.entity_weight = &om;
  if (kind == FRECSYS_KIND_WEIGHTED_V) {
    nuv.assign(nu->data(), nu->data() + nu->size());
    p.entity_reg = er.data();
    p.other_weight = nuv.data();
  }
  ctx.Solve(DeviceContext::USER, p);
  MatrixXf out = ctx.Get(DeviceContext::USER);
  VectorXf x(d);
  for (int j = 0; j < d; ++j) x[j] = out(0, j);
  return x;
}

}  // namespace detail
}  // namespace frecsys
