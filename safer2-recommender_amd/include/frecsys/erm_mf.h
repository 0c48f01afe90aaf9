// erm_mf.h -- ERM-MF on MI355X (reference erm_mf.h:34-611, same surface).
//
// SAFER2's solve loop with a constant dual weight omega = alpha that is
// never updated (erm_mf.h:53): StepU (FRECSYS_KIND_WEIGHTED_U, cached item
// Gramian), StepV (U^T diag(omega) U, nu = omega/|H_u|,
// FRECSYS_KIND_WEIGHTED_V with the tail quirk), item_gramian_ = V^T V,
// ComputeUserLoss (erm_mf.h:257-301).
#pragma once

#include <vector>

#include "frecsys/model_base.h"
#include "frecsys/safer2.h"

namespace frecsys {

class ERMMFRecommender : public detail::DeviceModel {
 public:
  ERMMFRecommender(int embedding_dim, int num_users, int num_items, float reg,
                   float unobserved_weight, float stdev, float alpha, bool use_cg,
                   float cg_error_tolerance, int cg_max_iterations,
                   const DeviceOptions& opts = DeviceOptions::FromEnv())
      : DeviceModel(embedding_dim, num_users, num_items, stdev, opts) {
    if (use_cg)  // BiCGSTAB path (erm_mf.h:138-145): not built
      LOG(FATAL) << "use_cg is not supported by the MI355X solve loop (LLT path only)";
    (void)cg_error_tolerance;
    (void)cg_max_iterations;
    regularization_ = reg;
    unobserved_weight_ = unobserved_weight;
    alpha_ = alpha;
    dual_weight_ = VectorXf::Constant(num_users, alpha);
    user_loss_ = VectorXf::Zero(num_users);
    user_history_size_ = VectorXf::Zero(num_users);
    item_reg_ = VectorXf::Zero(num_items);
    dev_->Gramian(DeviceContext::ITEM);  // item_gramian_ = V^T V, erm_mf.h:51
  }

  VectorXf Score(const int, const SpVector&) override {
    throw("Function 'Score' is not implemented");
  }

  static const VectorXf ProjectU(const SpVector& h, const MatrixXf& X, const MatrixXf& G,
                                 const float reg, const float w, const float weight, bool use_cg,
                                 const float = 1e-10, const int = 100) {
    return SAFER2Recommender::ProjectU(h, X, G, reg, w, weight, use_cg);
  }
  static const VectorXf ProjectV(const SpVector& h, const MatrixXf& X, const MatrixXf& G,
                                 const float reg, const float w, const VectorXf& dw, bool use_cg,
                                 const float = 1e-10, const int = 100) {
    return SAFER2Recommender::ProjectV(h, X, G, reg, w, dw, use_cg);
  }

  EvaluationResult EvaluateDataset(const VectorXi& k_list, const VectorXf& alpha_list,
                                   const Dataset& data, const SpMatrix& eval_by_user) override {
    frecsys_solve_params p = solve_params(FRECSYS_KIND_WEIGHTED_U, regularization_,
                                          unobserved_weight_);  // omega = 1 (erm_mf.h:235-244)
    return FoldInEvaluate(k_list, alpha_list, data, eval_by_user, p);
  }

  void Train(const Dataset& data) override {
    dev_->LoadTraining(data);
    PrintWeightedLosses(data, regularization_, unobserved_weight_, alpha_);  // erm_mf.h:258
    frecsys_solve_params pu = solve_params(FRECSYS_KIND_WEIGHTED_U, regularization_,
                                           unobserved_weight_);
    pu.entity_weight = dual_weight_.data();
    // residual norms (print_residual_stats, erm_mf.h:434-448, 508-512): U
    // and V against their pre-step values, on the device from snapshots
    if (print_residualstats_) dev_->Snapshot(DeviceContext::USER);
    dev_->Solve(DeviceContext::USER, pu);  // erm_mf.h:259-267
    const float residual_U = print_residualstats_ ? dev_->SnapshotResidual(DeviceContext::USER) : 0.0f;
    std::vector<float> nu((size_t)num_users_);
    for (int64_t u = 0; u < num_users_; ++u) nu[u] = dual_weight_[u] / user_history_size_[u];
    dev_->Gramian(DeviceContext::USER, dual_weight_.data(), ++weight_epoch_);
    frecsys_solve_params pv = solve_params(FRECSYS_KIND_WEIGHTED_V, regularization_,
                                           unobserved_weight_);
    pv.alpha = alpha_;
    pv.entity_reg = item_reg_.data();
    pv.other_weight = nu.data();
    if (print_residualstats_) dev_->Snapshot(DeviceContext::ITEM);
    dev_->Solve(DeviceContext::ITEM, pv);  // erm_mf.h:269-271
    const float residual_V = print_residualstats_ ? dev_->SnapshotResidual(DeviceContext::ITEM) : 0.0f;
    dev_->Gramian(DeviceContext::ITEM);    // erm_mf.h:273-274
    dev_->UserLoss(DeviceContext::USER, unobserved_weight_, true, user_loss_.data());
    VectorXf wl(num_users_);
    for (int64_t u = 0; u < num_users_; ++u) wl[u] = dual_weight_[u] * user_loss_[u];
    LOG(INFO) << "Weighted Loss: " << wl.mean();  // erm_mf.h:277-278
    if (print_varstats_) {
      PrintVarStats(alpha_);
      LOG(INFO) << format("Min: {0:.3f}, Mean: {1:.3f}, Max: {2:.3f}", dual_weight_.minCoeff(),
                          dual_weight_.mean(), dual_weight_.maxCoeff());
    }
    if (print_residualstats_)  // erm_mf.h:297-300
      LOG(INFO) << format("U residual: {0}, V residual: {1}", residual_U, residual_V);
  }

  // Initialize (erm_mf.h:573-587).
  void Initialize(const Dataset& data) {
    dev_->LoadTraining(data);
    dev_->Gramian(DeviceContext::ITEM);
    dev_->UserLoss(DeviceContext::USER, unobserved_weight_, true, user_loss_.data());
    ComputeHistoryStats(data);
  }

  float GetMeanWeight() const { return dual_weight_.mean(); }

 protected:
  void OnEmbeddingsSet() override { dev_->Gramian(DeviceContext::ITEM); }

 private:
  float regularization_;
  float unobserved_weight_;
  float alpha_;
  uint64_t weight_epoch_ = 0;
};

}  // namespace frecsys
