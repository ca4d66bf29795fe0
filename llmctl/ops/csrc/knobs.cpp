// Native side of llmctl.config.knobs: kernel-selection knobs the HIP launchers consult
// (flash-attention split / priority / wave count, dK/dV schedule, decode splits, decode skinny
// GEMM version).  Python pushes the resolved PerfKnobs here once (llmctl.config.knobs.apply);
// a launcher reads knob("name", default) -- no environment lookups on the hot path.
#include <cstdint>
#include <map>
#include <mutex>
#include <string>

namespace llmctl {
namespace {
std::mutex& mu() {
  static std::mutex m;
  return m;
}
std::map<std::string, int64_t>& table() {
  static std::map<std::string, int64_t> t;
  return t;
}
}  // namespace

int64_t knob(const char* name, int64_t dflt) {
  std::lock_guard<std::mutex> lk(mu());
  auto it = table().find(name);
  return it == table().end() ? dflt : it->second;
}

void set_knob(const std::string& name, int64_t value) {
  std::lock_guard<std::mutex> lk(mu());
  table()[name] = value;
}

void clear_knobs() {
  std::lock_guard<std::mutex> lk(mu());
  table().clear();
}
}  // namespace llmctl
