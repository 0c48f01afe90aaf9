// ials.h -- iALS on MI355X (reference ials.h:37-445, same public surface).
//
// Train() is the reference sequence (ials.h:187-224): U step against V
// (Gramian V^T V, per-user Project), V step against the new U, optional
// ComputeLosses diagnostics, ComputeUserLoss.  The per-entity work and the
// Gramians run in libfrecsys_hip.so (FRECSYS_KIND_IALS); U, V and G stay in
// HBM across epochs.
#pragma once

#include <chrono>
#include <string>

#include "frecsys/model_base.h"

namespace frecsys {

class IALSRecommender : public detail::DeviceModel {
 public:
  IALSRecommender(int embedding_dim, int num_users, int num_items, float reg, float reg_exp,
                  float unobserved_weight, float stdev, float alpha, bool use_cg,
                  float cg_error_tolerance, int cg_max_iterations,
                  const DeviceOptions& opts = DeviceOptions::FromEnv())
      : DeviceModel(embedding_dim, num_users, num_items, stdev, opts) {
    if (use_cg)  // Eigen ConjugateGradient path (ials.h:133-139): not built
      LOG(FATAL) << "use_cg is not supported by the MI355X solve loop (LLT path only)";
    (void)cg_error_tolerance;
    (void)cg_max_iterations;
    regularization_ = reg;
    regularization_exp_ = reg_exp;
    unobserved_weight_ = unobserved_weight;
    alpha_ = alpha;
    user_loss_ = VectorXf::Zero(num_users);
  }

  VectorXf Score(const int, const SpVector&) override {
    throw("Function 'Score' is not implemented");  // ials.h:65-68
  }

  // Per-entity solve (ials.h:88-144) on the GPU; `reg` is the final lambda.
  static const VectorXf Project(const SpVector& user_history, const MatrixXf& item_embeddings,
                                const MatrixXf& gramian, const float reg,
                                const float unobserved_weight, bool use_cg,
                                const float cg_error_tolerance = 1e-10,
                                const int cg_max_iterations = 100) {
    (void)cg_error_tolerance;
    (void)cg_max_iterations;
    if (use_cg) LOG(FATAL) << "use_cg is not supported";
    return detail::ProjectOnDevice(FRECSYS_KIND_IALS, user_history, item_embeddings, gramian,
                                   reg, unobserved_weight, 1.0f, nullptr);
  }

  EvaluationResult EvaluateDataset(const VectorXi& k_list, const VectorXf& alpha_list,
                                   const Dataset& data, const SpMatrix& eval_by_user) override {
    dev_->Gramian(DeviceContext::ITEM);  // Step's V^T V (ials.h:321)
    return FoldInEvaluate(k_list, alpha_list, data, eval_by_user, params());
  }

  void Train(const Dataset& data) override {
    dev_->LoadTraining(data);
    dev_->Gramian(DeviceContext::ITEM);            // ials.h:321 (V^T V)
    dev_->Solve(DeviceContext::USER, params());    // ials.h:188-193
    dev_->Gramian(DeviceContext::USER);            // ials.h:321 (U^T U)
    dev_->Solve(DeviceContext::ITEM, params());    // ials.h:196-201
    ComputeLosses(data);                           // ials.h:203
    dev_->Gramian(DeviceContext::ITEM);            // ials.h:371
    const bool need = print_varstats_;
    dev_->UserLoss(DeviceContext::USER, unobserved_weight_, false,
                   need ? user_loss_.data() : nullptr);  // ials.h:205-206
    if (print_varstats_) PrintVarStats(alpha_);
    if (print_residualstats_)
      LOG(INFO) << format("U residual: {0}, V residual: {1}", 0.0f, 0.0f);
  }

  // ComputeLosses (ials.h:226-305), diagnostics only.
  void ComputeLosses(const Dataset& data) {
    if (!print_trainstats_) return;
    const auto t0 = std::chrono::steady_clock::now();
    const LossParts lp = ComputeLossParts(data);
    const Csr& uc = data.user_csr();
    const Csr& ic = data.item_csr();
    double loss_reg = 0.0, reg_user_now = 0.0, reg_item_now = 0.0;
    for (int64_t u = 0; u < uc.rows(); ++u) {
      if (!uc.len(u)) continue;
      const double n2 = lp.user_norm2[u];
      loss_reg += n2 * RegularizationValue((int)uc.len(u), (int)num_items_);
      reg_user_now += n2;
    }
    for (int64_t i = 0; i < ic.rows(); ++i) {
      if (!ic.len(i)) continue;
      const double n2 = lp.item_norm2[i];
      loss_reg += n2 * RegularizationValue((int)ic.len(i), (int)num_users_);
      reg_item_now += n2;
    }
    const float loss =
        (float)(lp.observed + unobserved_weight_ * lp.unobserved + loss_reg);
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

  // RegularizationValue (ials.h:310-315).
  const float RegularizationValue(int history_size, int num_choices) const {
    return regularization_ *
           std::pow(history_size + unobserved_weight_ * num_choices, regularization_exp_);
  }

 private:
  frecsys_solve_params params() const {
    frecsys_solve_params p = solve_params(FRECSYS_KIND_IALS, regularization_, unobserved_weight_);
    p.reg_exp = regularization_exp_;
    return p;
  }

  float regularization_;
  float regularization_exp_;
  float unobserved_weight_;
  float alpha_;
};

}  // namespace frecsys
