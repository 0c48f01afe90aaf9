// model_dump -- test driver for the C++ model classes (the product's host
// layer).  Builds one of the four models with a fixed seed, optionally
// Initialize()s it, runs E Train() epochs on a training CSV and writes
//   int64 n_users, n_items, dim; float U[n_users*dim]; float V[n_items*dim];
//   float user_loss[n_users]; float dual_weight[n_users]; float xi;
//   float mean_weight_per_epoch[E]; then E x (fold-in NDCG@20) if asked
// to the output file.  tests/test_models_gpu.py compares it with the CPU
// oracle's Train() trajectory.
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "frecsys/cvar_mf.h"
#include "frecsys/erm_mf.h"
#include "frecsys/ials.h"
#include "frecsys/safer2.h"

int main(int argc, char** argv) {
  if (argc < 13) {
    fprintf(stderr,
            "usage: model_dump model dim epochs seed train.csv out.bin reg w alpha bandwidth "
            "stepsize epan [use_snr sampling_ratio [test_tr test_te]]\n");
    return 2;
  }
  const std::string model = argv[1];
  const int dim = atoi(argv[2]), epochs = atoi(argv[3]);
  const long seed = atol(argv[4]);
  frecsys::Dataset train(argv[5]);
  const std::string out = argv[6];
  const float reg = atof(argv[7]), w = atof(argv[8]), alpha = atof(argv[9]),
              bw = atof(argv[10]), eta = atof(argv[11]);
  const bool epan = atoi(argv[12]) != 0;
  const bool use_snr = argc >= 15 && atoi(argv[13]) != 0;
  const float sampling_ratio = argc >= 15 ? (float)atof(argv[14]) : 0.1f;
  frecsys::DeviceOptions o;
  o.seed = seed;
  const int nu = train.max_user() + 1, ni = train.max_item() + 1;
  frecsys::detail::DeviceModel* m = nullptr;
  frecsys::SAFER2Recommender* s2 = nullptr;
  frecsys::ERMMFRecommender* erm = nullptr;
  frecsys::CVaRMFRecommender* cv = nullptr;
  if (model == "ials") {
    // MODEL_DUMP_REG_EXP: iALS l2_reg_exp (default 1, run_model.cc:143-145)
    const char* re = getenv("MODEL_DUMP_REG_EXP");
    m = new frecsys::IALSRecommender(dim, nu, ni, reg, re ? (float)atof(re) : 1.0f, w, 0.1f, alpha,
                                     false, 1e-10, 100, o);
  } else if (model == "safer2") {
    s2 = new frecsys::SAFER2Recommender(dim, nu, ni, reg, w, bw, alpha, 0.1f, 5, 1, epan, use_snr,
                                        sampling_ratio, false, 1e-10, 100, o);
    m = s2;
  } else if (model == "erm_mf") {
    erm = new frecsys::ERMMFRecommender(dim, nu, ni, reg, w, 0.1f, alpha, false, 1e-10, 100, o);
    m = erm;
  } else if (model == "cvar_mf") {
    cv = new frecsys::CVaRMFRecommender(dim, nu, ni, reg, w, alpha, eta, 0.1f, o);
    m = cv;
  } else {
    return 3;
  }
  m->SetPrintTrainStats(false);
  // MODEL_DUMP_RESIDUAL_STATS=1: --print_residual_stats (the residual-norm
  // log lines, tests/test_models_gpu.py::test_residual_stats_match_oracle)
  if (const char* rs = getenv("MODEL_DUMP_RESIDUAL_STATS")) m->SetPrintResidualStats(atoi(rs) != 0);
  if (s2) s2->Initialize(train);
  if (erm) erm->Initialize(train);
  if (cv) cv->Initialize(train);
  std::vector<float> mean_w;
  std::vector<float> ndcg20;
  for (int e = 0; e < epochs; ++e) {
    m->Train(train);
    mean_w.push_back(s2 ? s2->GetMeanWeight() : erm ? erm->GetMeanWeight()
                                                     : cv ? cv->GetMeanWeight() : 0.0f);
  }
  if (argc >= 17) {
    frecsys::Dataset tr(argv[15]), te(argv[16]);
    frecsys::VectorXi k(5);
    k << 5, 10, 20, 50, 100;
    frecsys::VectorXf a(9);
    a << 0.1f, 0.2f, 0.3f, 0.4f, 0.5f, 0.6f, 0.7f, 0.8f, 0.9f;
    frecsys::EvaluationResult r = m->EvaluateDataset(k, a, tr, te.by_user());
    r.show();
    ndcg20.push_back(r.ndcg.colwise().mean()[2]);
  }
  const frecsys::MatrixXf U = m->user_embedding(), V = m->item_embedding();
  frecsys::VectorXf loss = m->user_loss();
  frecsys::VectorXf dw = s2 ? s2->dual_weight() : cv ? cv->dual_weight() : frecsys::VectorXf::Zero(nu);
  float xi = s2 ? s2->xi() : cv ? cv->xi() : 0.0f;
  FILE* f = fopen(out.c_str(), "wb");
  int64_t hdr[3] = {nu, ni, dim};
  fwrite(hdr, sizeof(hdr), 1, f);
  fwrite(U.data(), sizeof(float), (size_t)nu * dim, f);
  fwrite(V.data(), sizeof(float), (size_t)ni * dim, f);
  fwrite(loss.data(), sizeof(float), (size_t)nu, f);
  fwrite(dw.data(), sizeof(float), (size_t)nu, f);
  fwrite(&xi, sizeof(float), 1, f);
  fwrite(mean_w.data(), sizeof(float), mean_w.size(), f);
  fwrite(ndcg20.data(), sizeof(float), ndcg20.size(), f);
  fclose(f);
  delete m;
  return 0;
}
