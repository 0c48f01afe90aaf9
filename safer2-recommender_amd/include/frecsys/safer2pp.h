// safer2pp.h -- SAFER2++ on MI355X (reference safer2pp.h:34-944, same
// public surface).
//
// SAFER2's primal-dual scheme with the iALS++ subspace solver: per
// primal-dual iteration the dual weights of every user (safer2pp.h:839-862),
// then per column block the weighted user block Step (ProjectU, Gramian of
// the items) and the weighted item block Step (ProjectV, rows weighted by
// nu_u = omega_u/|H_u|, Gramian U^T diag(omega) U) -- safer2pp.h:288-349 --
// each one launch of frecsys_pp_step with the prediction vector resident on
// the device; the losses, xi and the diagnostics are SAFER2's.
#pragma once

#include <algorithm>
#include <cmath>
#include <vector>

#include "frecsys/safer2.h"

namespace frecsys {

class SAFER2ppRecommender : public SAFER2Recommender {
 public:
  SAFER2ppRecommender(int embedding_dim, int num_users, int num_items, float reg,
                      float unobserved_weight, float bandwidth, float alpha, float stdev,
                      int xi_iterations, int pd_iterations, bool use_epanechnikov, bool use_snr,
                      float sampling_ratio, int block_size,
                      const DeviceOptions& opts = DeviceOptions::FromEnv())
      : SAFER2Recommender(embedding_dim, num_users, num_items, reg, unobserved_weight, bandwidth,
                          alpha, stdev, xi_iterations, pd_iterations, use_epanechnikov, use_snr,
                          sampling_ratio, false, 1e-10f, 100, opts) {
    if (block_size < 1 || block_size > 128)
      LOG(FATAL) << "block_size must be in [1, 128] on the MI355X build (got " << block_size
                 << ")";
    block_size_ = block_size;
  }

  // Fold-in: 8 epochs of weighted (omega = 1) user block steps from zero
  // embeddings (safer2pp.h:220-286), then GPU scoring + top-K.
  EvaluationResult EvaluateDataset(const VectorXi& k_list, const VectorXf& alpha_list,
                                   const Dataset& data, const SpMatrix& eval_by_user) override {
    std::vector<int32_t> ids;
    Csr csr;
    data.compact_users(&ids, &csr);
    dev_->LoadEval(csr);
    dev_->ZeroEval(dim_);
    const frecsys_solve_params p = u_params(false);
    for (int e = 0; e < 8; ++e) {
      dev_->PPPredict(DeviceContext::EVAL);
      for (int start = 0; start < dim_; start += block_size_) {
        const int end = std::min(start + block_size_, dim_);
        dev_->Gramian(DeviceContext::ITEM);
        dev_->PPStep(DeviceContext::EVAL, start, end, p);
      }
    }
    return RankEval(k_list, alpha_list, ids, eval_by_user);
  }

  void Train(const Dataset& data) override {
    dev_->PPLoad(data);
    PrintLosses(data);                                      // safer2pp.h:289
    dev_->PPPredict(DeviceContext::USER);                   // safer2pp.h:291-297
    for (int t = 0; t < pd_iterations_; ++t) {
      const float residual_z = ComputeAllUserWeights();     // safer2pp.h:301-302
      std::vector<float> nu((size_t)num_users_);
      for (int64_t u = 0; u < num_users_; ++u) nu[u] = dual_weight_[u] / user_history_size_[u];
      ++weight_epoch_;
      double residual_U = 0, residual_V = 0;
      for (int start = 0; start < dim_; start += block_size_) {  // safer2pp.h:303-318
        const int end = std::min(start + block_size_, dim_);
        dev_->Gramian(DeviceContext::ITEM);
        residual_U += dev_->PPStep(DeviceContext::USER, start, end, u_params(true));
        dev_->Gramian(DeviceContext::USER, dual_weight_.data(), weight_epoch_);
        frecsys_solve_params pv = solve_params(FRECSYS_KIND_WEIGHTED_V, regularization_,
                                               unobserved_weight_);
        pv.alpha = alpha_;
        pv.entity_reg = item_reg_.data();
        pv.other_weight = nu.data();
        residual_V += dev_->PPStep(DeviceContext::ITEM, start, end, pv);
      }
      dev_->Gramian(DeviceContext::ITEM);                   // safer2pp.h:319-320
      dev_->UserLoss(DeviceContext::USER, unobserved_weight_, true, user_loss_.data());
      VectorXf wl(num_users_);
      for (int64_t u = 0; u < num_users_; ++u) wl[u] = dual_weight_[u] * user_loss_[u];
      LOG(INFO) << "Weighted Loss: " << wl.mean();          // safer2pp.h:324-325
      if (print_varstats_) {
        PrintVarStats(alpha_);
        LOG(INFO) << format("Min: {0:.3f}, Mean: {1:.3f}, Max: {2:.3f}", dual_weight_.minCoeff(),
                            dual_weight_.mean(), dual_weight_.maxCoeff());
      }
      if (print_residualstats_)
        LOG(INFO) << format("U residual: {0}, V residual: {1}, z residual: {2}",
                            (float)std::sqrt(residual_U), (float)std::sqrt(residual_V),
                            residual_z);
    }
    const float xi = ComputeXi(user_loss_, prev_xi_, xi_iterations_);  // safer2pp.h:352-354
    LOG(INFO) << "Xi:" << xi;
    prev_xi_ = xi;
  }

 private:
  // ComputeUserWeights (safer2pp.h:839-862): every user, history or not.
  float ComputeAllUserWeights() {
    VectorXf prev;
    if (print_residualstats_) prev = dual_weight_;
    for (int64_t u = 0; u < num_users_; ++u)
      dual_weight_[u] = smoother_.Weight(user_loss_[u], prev_xi_);
    if (!print_residualstats_) return 0.0f;
    double s = 0.0;
    for (int64_t u = 0; u < num_users_; ++u) {
      const double d = (double)dual_weight_[u] - prev[u];
      s += d * d;
    }
    return (float)std::sqrt(s);
  }

  int block_size_;
};

}  // namespace frecsys
