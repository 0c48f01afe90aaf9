// logging.h -- glog-compatible LOG(...) lines and an fmt-style formatter.
//
// The reference logs through glog (`LOG(INFO) << ...`) with fmt::format
// payloads (e.g. run_model.cc:266 "Epoch: {0}, Timer: Train={1}",
// evaluation.h:41 "{0}@{1}={2:.4f}").  Neither library is a dependency
// here; these two small pieces keep the line formats byte-compatible:
//   I<mmdd> <hh:mm:ss.uuuuuu> <tid> <file>:<line>] <message>
// and the positional `{N}` / `{N:.Kf}` replacement fields.
#pragma once

#include <sys/syscall.h>
#include <sys/time.h>
#include <unistd.h>

#include <charconv>
#include <cstdio>
#include <cstdlib>
#include <ctime>
#include <sstream>
#include <string>
#include <type_traits>
#include <vector>

namespace frecsys {
namespace logging {

enum Severity { INFO = 0, WARNING = 1, ERROR = 2, FATAL = 3 };

class Line {
 public:
  Line(Severity s, const char* file, int line) : sev_(s), file_(file), line_(line) {}
  ~Line() {
    static const char kSev[] = "IWEF";
    struct timeval tv;
    gettimeofday(&tv, nullptr);
    struct tm tm;
    localtime_r(&tv.tv_sec, &tm);
    const char* base = file_;
    for (const char* p = file_; *p; ++p)
      if (*p == '/') base = p + 1;
    char pre[128];
    snprintf(pre, sizeof(pre), "%c%02d%02d %02d:%02d:%02d.%06ld %ld %s:%d] ", kSev[sev_],
             tm.tm_mon + 1, tm.tm_mday, tm.tm_hour, tm.tm_min, tm.tm_sec, (long)tv.tv_usec,
             (long)syscall(SYS_gettid), base, line_);
    std::string out = pre + os_.str() + "\n";
    fwrite(out.data(), 1, out.size(), stderr);
    fflush(stderr);
    if (sev_ == FATAL) abort();
  }
  template <typename T>
  Line& operator<<(const T& v) {
    os_ << v;
    return *this;
  }

 private:
  Severity sev_;
  const char* file_;
  int line_;
  std::ostringstream os_;
};

}  // namespace logging

// ---- fmt-style positional formatting ------------------------------------
namespace detail {

inline std::string shortest(double x, bool is_float) {
  char buf[64];
  std::to_chars_result r = is_float ? std::to_chars(buf, buf + sizeof(buf), (float)x)
                                    : std::to_chars(buf, buf + sizeof(buf), x);
  return std::string(buf, r.ptr);
}

template <typename T>
std::string fmt_one(const T& v, const std::string& spec) {
  if constexpr (std::is_floating_point_v<T>) {
    if (!spec.empty() && spec[0] == '.' && spec.back() == 'f') {
      char buf[64];
      snprintf(buf, sizeof(buf), ("%" + spec).c_str(), (double)v);
      return buf;
    }
    return shortest((double)v, std::is_same_v<T, float>);
  } else if constexpr (std::is_integral_v<T>) {
    return std::to_string(v);
  } else {
    std::ostringstream os;
    os << v;
    return os.str();
  }
}

}  // namespace detail

// format("{0}@{1}={2:.4f}", "Rec", 5, 0.25f) -> "Rec@5=0.2500"
template <typename... Args>
std::string format(const std::string& f, const Args&... args) {
  std::vector<std::string (*)(const void*, const std::string&)> fns;
  std::vector<const void*> ptrs;
  (fns.push_back([](const void* p, const std::string& s) {
     return detail::fmt_one(*static_cast<const Args*>(p), s);
   }),
   ...);
  (ptrs.push_back(static_cast<const void*>(&args)), ...);
  std::string out;
  size_t next = 0;
  for (size_t i = 0; i < f.size(); ++i) {
    if (f[i] == '{' && i + 1 < f.size() && f[i + 1] == '{') {
      out += '{';
      ++i;
    } else if (f[i] == '}' && i + 1 < f.size() && f[i + 1] == '}') {
      out += '}';
      ++i;
    } else if (f[i] == '{') {
      size_t j = f.find('}', i);
      std::string field = f.substr(i + 1, j - i - 1);
      std::string idx = field, spec;
      size_t colon = field.find(':');
      if (colon != std::string::npos) {
        idx = field.substr(0, colon);
        spec = field.substr(colon + 1);
      }
      size_t k = idx.empty() ? next++ : (size_t)std::stoul(idx);
      if (k < fns.size()) out += fns[k](ptrs[k], spec);
      i = j;
    } else {
      out += f[i];
    }
  }
  return out;
}

}  // namespace frecsys

#ifndef LOG
#define LOG(sev) ::frecsys::logging::Line(::frecsys::logging::sev, __FILE__, __LINE__)
#endif

// The reference spells the formatter fmt::format (run_model.cc:266).
namespace fmt {
using ::frecsys::format;
}
