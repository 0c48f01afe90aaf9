// run_model -- reference-compatible CLI (tools/run_model.cc of the
// reference): same flags and defaults (run_model.cc:129-230), same model
// factory (run_model.cc:43-123), same epoch loop and log lines
// ("Epoch: {e}, Timer: Train={ms}", run_model.cc:258-270), final
// "Validation Results" evaluation (run_model.cc:271-272).  The models are
// the MI355X ones (include/frecsys/*.h over libfrecsys_hip.so).
//
// Added flags: --seed (deterministic init; the reference seeds from
// std::random_device), --device (HIP ordinal), --parity_quirks (0/1,
// SURVEY App. A.1).  One process per GPU for multi-GPU runs: WORLD_SIZE /
// RANK / LOCAL_RANK from the environment (torchrun-style), RCCL id through
// FRECSYS_COMM_FILE.  iALS++ / SAFER2++ (ialspp.h, safer2pp.h) run on the
// GPU block-step kernels.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <string>
#include <sys/stat.h>

#include "frecsys/factory.h"

namespace {

struct Flag {
  std::string value;
  bool required = false;
  bool set = false;
};

class Flags {
 public:
  void add(const std::string& names, const std::string& dflt, bool required = false) {
    std::string canon;
    size_t start = 0;
    while (start <= names.size()) {
      size_t comma = names.find(',', start);
      std::string n = names.substr(start, comma == std::string::npos ? std::string::npos
                                                                      : comma - start);
      if (canon.empty() || n.rfind("--", 0) == 0) canon = n;
      alias_.push_back(n);
      if (comma == std::string::npos) break;
      start = comma + 1;
    }
    for (size_t i = alias_.size(); i-- > 0;) {
      if (alias_map_.count(alias_[i])) break;
      alias_map_[alias_[i]] = canon;
    }
    flags_[canon] = Flag{dflt, required, false};
  }
  bool parse(int argc, char** argv) {
    for (int i = 1; i < argc; ++i) {
      std::string a = argv[i], v;
      size_t eq = a.find('=');
      if (eq != std::string::npos) {
        v = a.substr(eq + 1);
        a = a.substr(0, eq);
      } else if (i + 1 < argc) {
        v = argv[++i];
      } else {
        fprintf(stderr, "%s: missing value\n", a.c_str());
        return false;
      }
      auto it = alias_map_.find(a);
      if (it == alias_map_.end()) {
        fprintf(stderr, "The following argument was not expected: %s\n", a.c_str());
        return false;
      }
      flags_[it->second].value = v;
      flags_[it->second].set = true;
    }
    for (auto& kv : flags_)
      if (kv.second.required && !kv.second.set) {
        fprintf(stderr, "%s is required\n", kv.first.c_str());
        return false;
      }
    return true;
  }
  std::string str(const std::string& n) const { return flags_.at(n).value; }
  int i(const std::string& n) const { return std::atoi(str(n).c_str()); }
  float f(const std::string& n) const { return (float)std::atof(str(n).c_str()); }
  bool b(const std::string& n) const {
    std::string v = str(n);
    std::transform(v.begin(), v.end(), v.begin(), ::tolower);
    return v == "1" || v == "true" || v == "on" || v == "yes";
  }

 private:
  std::vector<std::string> alias_;
  std::map<std::string, std::string> alias_map_;
  std::map<std::string, Flag> flags_;
};

template <typename F>
void evaluate(int epoch, F recommender, frecsys::Dataset& exclude, frecsys::Dataset& test) {
  Eigen::VectorXi k_list = Eigen::VectorXi::Zero(5);
  Eigen::VectorXf alpha_list = Eigen::VectorXf::Zero(9);
  k_list << 5, 10, 20, 50, 100;
  alpha_list << 0.1f, 0.2f, 0.3f, 0.4f, 0.5f, 0.6f, 0.7f, 0.8f, 0.9f;
  frecsys::EvaluationResult metrics =
      recommender->EvaluateDataset(k_list, alpha_list, exclude, test.by_user());
  LOG(INFO) << "Epoch " << epoch << ":";
  metrics.show();
}

frecsys::ModelParams model_params(const Flags& a) {
  frecsys::ModelParams p;
  p.dim = a.i("--dim");
  p.l2_reg = a.f("--l2_reg");
  p.l2_reg_exp = a.f("--l2_reg_exp");
  p.uobs_weight = a.f("--uobs_weight");
  p.stdev = a.f("--stdev");
  p.alpha = a.f("--alpha");
  p.bandwidth = a.f("--bandwidth");
  p.stepsize = a.f("--stepsize");
  p.sampling_ratio = a.f("--sampling_ratio");
  p.cg_error_tolerance = a.f("--cg_error_tolerance");
  p.cg_max_iterations = a.i("--cg_max_iterations");
  p.use_cg = a.b("--use_cg");
  p.block_size = a.i("--block_size");
  p.xi_iterations = a.i("--xi_iterations");
  p.pd_iterations = a.i("--pd_iterations");
  p.use_epanechnikov = a.b("--use_epanechnikov");
  p.use_snr = a.b("--use_snr");
  p.print_train_stats = a.b("--print_train_stats");
  p.print_residual_stats = a.b("--print_residual_stats");
  p.print_var_stats = a.b("--print_var_stats");
  return p;
}

}  // namespace

int main(int argc, char* argv[]) {
  Flags app;  // run_model.cc:129-230
  app.add("--print_evaluation_stats", "false");
  app.add("-d,--dim", "8");
  app.add("--uobs_weight", "0.1");
  app.add("-r,--l2_reg", "0.002");
  app.add("--l2_reg_exp", "1.0");
  app.add("-s,--stdev", "0.1");
  app.add("--print_train_stats", "true");
  app.add("--print_test_results", "false");
  app.add("--print_residual_stats", "false");
  app.add("--print_var_stats", "false");
  app.add("--cg_error_tolerance", "1e-10");
  app.add("--cg_max_iterations", "100");
  app.add("--use_cg", "false");
  app.add("--block_size", "64");
  app.add("--alpha", "0.3");
  app.add("--bandwidth", "1.0");
  app.add("--stepsize", "0.1");
  app.add("--xi_iterations", "5");
  app.add("--sampling_ratio", "0.1");
  app.add("--pd_iterations", "1");
  app.add("--use_epanechnikov", "false");
  app.add("--use_snr", "false");
  app.add("-e,--epoch", "50");
  app.add("-n,--model_name", "", true);
  app.add("--train_data", "", true);
  app.add("--test_train_data", "", true);
  app.add("--test_test_data", "", true);
  app.add("--seed", "-1");
  app.add("--device", "-1");
  app.add("--parity_quirks", "1");
  if (!app.parse(argc, argv)) return 106;

  std::string model_name = app.str("--model_name");
  std::transform(model_name.begin(), model_name.end(), model_name.begin(), ::tolower);
  if (!frecsys::IsKnownModel(model_name)) {
    fprintf(stderr, "--model_name: %s not in {ials,ialspp,safer2,safer2pp,cvar_mf,erm_mf}\n",
            model_name.c_str());
    return 105;
  }
  for (const char* f : {"--train_data", "--test_train_data", "--test_test_data"}) {
    struct stat st;
    if (stat(app.str(f).c_str(), &st) != 0) {
      fprintf(stderr, "%s: File does not exist: %s\n", f, app.str(f).c_str());
      return 105;
    }
  }

  frecsys::Dataset train(app.str("--train_data"));
  frecsys::Dataset test_tr(app.str("--test_train_data"));
  frecsys::Dataset test_te(app.str("--test_test_data"));

  frecsys::DeviceOptions opts;
  opts.seed = std::atoll(app.str("--seed").c_str());
  opts.device = app.i("--device");
  opts.parity_quirks = app.b("--parity_quirks");
  frecsys::Recommender* recommender = frecsys::MakeRecommender(
      model_name, train.max_user() + 1, train.max_item() + 1, model_params(app), opts);
  setbuf(stdout, NULL);

  frecsys::InitializeRecommender(model_name, recommender, train);  // run_model.cc:246-257
  const int epochs = app.i("--epoch");
  const bool print_eval = app.b("--print_evaluation_stats");
  for (int epoch = 0; epoch < epochs; ++epoch) {
    auto t0 = std::chrono::steady_clock::now();
    recommender->Train(train);
    auto t1 = std::chrono::steady_clock::now();
    uint64_t train_time =
        std::chrono::duration_cast<std::chrono::milliseconds>(t1 - t0).count();
    LOG(INFO) << fmt::format("Epoch: {0}, Timer: Train={1}", epoch, train_time);
    if (print_eval) evaluate(epoch, recommender, test_tr, test_te);
  }
  LOG(INFO) << "Validation Results";
  evaluate(epochs, recommender, test_tr, test_te);
  delete recommender;
  return 0;
}
