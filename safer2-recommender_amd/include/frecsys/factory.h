// factory.h -- the model factory of run_model (reference run_model.cc:43-123)
// and its Initialize() dispatch (run_model.cc:246-257), shared by the CLI
// (tools/run_model.cc) and the model C-ABI (tools/model_capi.cc,
// include/frecsys_model.h).  ModelParams carries the run_model flags with
// the reference defaults (run_model.cc:129-230).
#pragma once

#include <string>

#include "frecsys/cvar_mf.h"
#include "frecsys/erm_mf.h"
#include "frecsys/ials.h"
#include "frecsys/ialspp.h"
#include "frecsys/safer2.h"
#include "frecsys/safer2pp.h"

namespace frecsys {

struct ModelParams {
  int dim = 8;
  float l2_reg = 0.002f;
  float l2_reg_exp = 1.0f;
  float uobs_weight = 0.1f;
  float stdev = 0.1f;
  float alpha = 0.3f;
  float bandwidth = 1.0f;
  float stepsize = 0.1f;
  float sampling_ratio = 0.1f;
  float cg_error_tolerance = 1e-10f;
  int cg_max_iterations = 100;
  bool use_cg = false;
  int block_size = 64;
  int xi_iterations = 5;
  int pd_iterations = 1;
  bool use_epanechnikov = false;
  bool use_snr = false;
  bool print_train_stats = true;
  bool print_residual_stats = false;
  bool print_var_stats = false;
};

inline bool IsKnownModel(const std::string& name) {
  for (const char* m : {"ials", "ialspp", "safer2", "safer2pp", "cvar_mf", "erm_mf"})
    if (name == m) return true;
  return false;
}

// get_model (run_model.cc:43-123) with the print flags applied.
inline Recommender* MakeRecommender(const std::string& name, int num_users, int num_items,
                                    const ModelParams& a, const DeviceOptions& o) {
  Recommender* r = nullptr;
  if (name == "ials") {
    r = new IALSRecommender(a.dim, num_users, num_items, a.l2_reg, a.l2_reg_exp, a.uobs_weight,
                            a.stdev, a.alpha, a.use_cg, a.cg_error_tolerance,
                            a.cg_max_iterations, o);
  } else if (name == "ialspp") {
    r = new IALSppRecommender(a.dim, num_users, num_items, a.l2_reg, a.l2_reg_exp,
                              a.uobs_weight, a.stdev, a.alpha, a.block_size, o);
  } else if (name == "safer2") {
    r = new SAFER2Recommender(a.dim, num_users, num_items, a.l2_reg, a.uobs_weight, a.bandwidth,
                              a.alpha, a.stdev, a.xi_iterations, a.pd_iterations,
                              a.use_epanechnikov, a.use_snr, a.sampling_ratio, a.use_cg,
                              a.cg_error_tolerance, a.cg_max_iterations, o);
  } else if (name == "safer2pp") {
    r = new SAFER2ppRecommender(a.dim, num_users, num_items, a.l2_reg, a.uobs_weight,
                                a.bandwidth, a.alpha, a.stdev, a.xi_iterations,
                                a.pd_iterations, a.use_epanechnikov, a.use_snr,
                                a.sampling_ratio, a.block_size, o);
  } else if (name == "erm_mf") {
    r = new ERMMFRecommender(a.dim, num_users, num_items, a.l2_reg, a.uobs_weight, a.stdev,
                             a.alpha, a.use_cg, a.cg_error_tolerance, a.cg_max_iterations, o);
  } else if (name == "cvar_mf") {
    r = new CVaRMFRecommender(a.dim, num_users, num_items, a.l2_reg, a.uobs_weight, a.alpha,
                              a.stepsize, a.stdev, o);
  } else {
    LOG(FATAL) << "model " << name << " is not part of this build";
  }
  r->SetPrintResidualStats(a.print_residual_stats);
  r->SetPrintVarStats(a.print_var_stats);
  r->SetPrintTrainStats(a.print_train_stats);
  return r;
}

// The Initialize(train) calls of run_model.cc:246-257 (iALS / iALS++ have none).
inline void InitializeRecommender(const std::string& name, Recommender* r, const Dataset& train) {
  if (name == "cvar_mf") static_cast<CVaRMFRecommender*>(r)->Initialize(train);
  if (name == "safer2") static_cast<SAFER2Recommender*>(r)->Initialize(train);
  if (name == "safer2pp") static_cast<SAFER2ppRecommender*>(r)->Initialize(train);
  if (name == "erm_mf") static_cast<ERMMFRecommender*>(r)->Initialize(train);
}

// The DeviceModel behind a factory-made recommender (every model class of
// this build derives from it).
inline detail::DeviceModel* AsDeviceModel(Recommender* r) {
  return static_cast<detail::DeviceModel*>(r);
}

}  // namespace frecsys
