// cvar_mf.h -- CVaR-MF on MI355X (reference cvar_mf.h:34-748, same surface).
//
// Train() (cvar_mf.h:276-330): hard 0/1 dual weights from the cached losses
// and the exact quantile xi; U_prev snapshot; one gradient step per user
// (FRECSYS_KIND_CVAR_GRAD_U: e - eta (A e - b) with the full matrix whose
// strict upper triangle lacks the observed term); one
// gradient step per item against the PRE-step U (snapshot, cvar_mf.h:282,
// 294) with U_prev^T diag(omega) U_prev; item_gramian_ = V^T V;
// ComputeUserLoss; xi = exact quantile.  Fold-in uses the LLT solve
// (ProjectU_eval, cvar_mf.h:182-229).
#pragma once

#include <algorithm>
#include <vector>

#include "frecsys/model_base.h"
#include "frecsys/safer2.h"

namespace frecsys {

class CVaRMFRecommender : public detail::DeviceModel {
 public:
  CVaRMFRecommender(int embedding_dim, int num_users, int num_items, float reg,
                    float unobserved_weight, float alpha, float stepsize, float stdev,
                    const DeviceOptions& opts = DeviceOptions::FromEnv())
      : DeviceModel(embedding_dim, num_users, num_items, stdev, opts) {
    regularization_ = reg;
    unobserved_weight_ = unobserved_weight;
    alpha_ = alpha;
    prev_xi_ = 0.0f;
    stepsize_ = stepsize;
    dual_weight_ = VectorXf::Constant(num_users, alpha);
    user_loss_ = VectorXf::Zero(num_users);
    user_history_size_ = VectorXf::Zero(num_users);
    item_reg_ = VectorXf::Zero(num_items);
    dev_->Gramian(DeviceContext::ITEM);
  }

  VectorXf Score(const int, const SpVector&) override {
    throw("Function 'Score' is not implemented");
  }

  static const VectorXf ProjectU_eval(const SpVector& h, const MatrixXf& X, const MatrixXf& G,
                                      const float reg, const float w, const float weight) {
    return SAFER2Recommender::ProjectU(h, X, G, reg, w, weight, false);
  }

  EvaluationResult EvaluateDataset(const VectorXi& k_list, const VectorXf& alpha_list,
                                   const Dataset& data, const SpMatrix& eval_by_user) override {
    frecsys_solve_params p = solve_params(FRECSYS_KIND_WEIGHTED_U, regularization_,
                                          unobserved_weight_);  // StepU_eval, omega = 1
    return FoldInEvaluate(k_list, alpha_list, data, eval_by_user, p);
  }

  void Train(const Dataset& data) override {
    dev_->LoadTraining(data);
    PrintWeightedLosses(data, regularization_, unobserved_weight_, alpha_);  // cvar_mf.h:277
    const Csr& uc = data.user_csr();
    VectorXf w_prev;
    if (print_residualstats_) w_prev = dual_weight_;
    for (int64_t u = 0; u < uc.rows() && u < num_users_; ++u)  // cvar_mf.h:597-642
      if (uc.len(u)) dual_weight_[u] = (float)((user_loss_[u] - prev_xi_) >= 0);
    // residual norms (print_residual_stats): z = (omega - omega_prev).norm()
    // (cvar_mf.h:637-640); StepU returns 0 (cvar_mf.h:472-473); V against
    // its pre-step value (cvar_mf.h:533-536), on the device from a snapshot
    const float residual_z = print_residualstats_ ? WeightResidual(dual_weight_, w_prev) : 0.0f;
    const float residual_U = 0.0f;
    dev_->Snapshot(DeviceContext::USER);  // user_embedding_prev, cvar_mf.h:282
    frecsys_solve_params pu = solve_params(FRECSYS_KIND_CVAR_GRAD_U, regularization_,
                                           unobserved_weight_);
    pu.stepsize = stepsize_;
    pu.entity_weight = dual_weight_.data();
    dev_->Solve(DeviceContext::USER, pu);  // cvar_mf.h:283-291
    std::vector<float> nu((size_t)num_users_);
    for (int64_t u = 0; u < num_users_; ++u) nu[u] = dual_weight_[u] / user_history_size_[u];
    dev_->Gramian(DeviceContext::USER, dual_weight_.data(), ++weight_epoch_, true);
    frecsys_solve_params pv = solve_params(FRECSYS_KIND_CVAR_GRAD_V, regularization_,
                                           unobserved_weight_);
    pv.alpha = alpha_;
    pv.stepsize = stepsize_;
    pv.from_snapshot = 1;
    pv.entity_reg = item_reg_.data();
    pv.other_weight = nu.data();
    if (print_residualstats_) dev_->Snapshot(DeviceContext::ITEM);
    dev_->Solve(DeviceContext::ITEM, pv);  // cvar_mf.h:293-295
    const float residual_V = print_residualstats_ ? dev_->SnapshotResidual(DeviceContext::ITEM) : 0.0f;
    dev_->Gramian(DeviceContext::ITEM);    // cvar_mf.h:297-298
    dev_->UserLoss(DeviceContext::USER, unobserved_weight_, true, user_loss_.data());
    VectorXf wl(num_users_);
    for (int64_t u = 0; u < num_users_; ++u) wl[u] = dual_weight_[u] * user_loss_[u];
    LOG(INFO) << "Weighted Loss: " << wl.mean();
    LOG(INFO) << "Mean weights: " << dual_weight_.mean();
    if (print_varstats_) {
      PrintVarStats(alpha_);
      LOG(INFO) << format("Min: {0:.3f}, Mean: {1:.3f}, Max: {2:.3f}", dual_weight_.minCoeff(),
                          dual_weight_.mean(), dual_weight_.maxCoeff());
    }
    if (print_residualstats_)  // cvar_mf.h:322-326
      LOG(INFO) << format("U residual: {0}, V residual: {1}, z residual: {2}", residual_U,
                          residual_V, residual_z);
    const float xi = ComputeXi(user_loss_);
    LOG(INFO) << "Xi:" << xi;
    prev_xi_ = xi;
  }

  // Exact quantile (cvar_mf.h:582-595): -nth_element(-loss)[N * alpha].
  float ComputeXi(const VectorXf& user_loss) {
    std::vector<float> vals((size_t)user_loss.size());
    for (int64_t i = 0; i < user_loss.size(); ++i) vals[i] = -user_loss[i];
    const size_t Q = (size_t)((float)vals.size() * alpha_);
    std::nth_element(vals.begin(), vals.begin() + Q, vals.end());
    LOG(INFO) << "Exact Quantile:" << -vals[Q];
    return -vals[Q];
  }

  // Initialize (cvar_mf.h:710-726): prev_xi_ is NOT updated there.
  void Initialize(const Dataset& data) {
    dev_->LoadTraining(data);
    dev_->Gramian(DeviceContext::ITEM);
    dev_->UserLoss(DeviceContext::USER, unobserved_weight_, true, user_loss_.data());
    ComputeHistoryStats(data);
  }

  float GetMeanWeight() const { return dual_weight_.mean(); }
  float xi() const { return prev_xi_; }
  const VectorXf& dual_weight() const { return dual_weight_; }

 protected:
  void OnEmbeddingsSet() override { dev_->Gramian(DeviceContext::ITEM); }

 private:
  float regularization_;
  float unobserved_weight_;
  float alpha_;
  float prev_xi_;
  float stepsize_;
  uint64_t weight_epoch_ = 0;
};

}  // namespace frecsys
