// lamm_knobs.cpp -- the LAMM_* switches (lamm_knobs.h), read once per load / reload.
#include "lamm_knobs.h"

#include <atomic>
#include <cstdlib>
#include <cstring>

namespace lamm {
namespace {

int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e && *e ? atoi(e) : dflt;
}
// "0" turns a default-on switch off
bool env_off(const char* name) {
  const char* e = getenv(name);
  return e && e[0] == '0';
}
// "1" turns a default-off switch on
bool env_on(const char* name) {
  const char* e = getenv(name);
  return e && e[0] == '1';
}

Knobs* read_env() {
  auto* k = new Knobs();
  if (const char* e = getenv("LAMM_GEMM_PATH")) {
    if (!strcmp(e, "i8") || !strcmp(e, "1")) k->gemm_path = 1;
    if (!strcmp(e, "fp6") || !strcmp(e, "0")) k->gemm_path = 0;
    if (!strcmp(e, "dq16") || !strcmp(e, "2")) k->gemm_path = 2;
  }
  k->gemv_max_n = env_int("LAMM_GEMV_MAX_N", -1);
  k->dense_gemm = !env_off("LAMM_DENSE_GEMM");
  k->kq_gemm = !env_off("LAMM_KQ_GEMM");
  k->fp6_split = env_int("LAMM_FP6_SPLIT", 0);
  k->fp6_sub = env_int("LAMM_FP6_SUB", -1);
  k->fp6_fused_reduce = env_on("LAMM_FP6_FUSED_REDUCE");
  k->fp6_wj = env_int("LAMM_FP6_WJ", 2);
  k->fp6_av = !env_off("LAMM_FP6_AV");
  k->fp6_kv_p = env_int("LAMM_FP6_KV_P", 0);
  k->i8_split = env_int("LAMM_I8_SPLIT", 0);
  k->dense_split = env_int("LAMM_DENSE_SPLIT", 0);
  k->kq_split = env_int("LAMM_KQ_SPLIT", 0);
  k->kq_variant = env_int("LAMM_KQ_VARIANT", 0);
  k->gemv_variant = env_int("LAMM_GEMV_VARIANT", 0);
  k->gemv_rpw = env_int("LAMM_GEMV_RPW", -1);
  k->gemv_laneb = env_on("LAMM_GEMV_LANEB");

  k->opt_level = env_int("LAMM_OPT_LEVEL", 3);
  k->device = env_int("LAMM_HIP_DEVICE", -1);
  if (const char* e = getenv("LAMM_HIP_DEVICES")) strncpy(k->devices, e, sizeof k->devices - 1);
  k->stats = env_int("LAMM_HIP_STATS", 0) > 0;
  k->stats_sync = env_int("LAMM_HIP_STATS", 0) == 2;
  if (const char* e = getenv("LAMM_HIP_CACHE_GB")) k->cache_gb = atof(e);
  k->pinned = !env_off("LAMM_HIP_PINNED");
  k->views = env_on("LAMM_HIP_VIEWS") ? 1 : env_off("LAMM_HIP_VIEWS") ? 0 : -1;
  k->extra_types = !env_off("LAMM_HIP_EXTRA_TYPES");
  k->gpu_quant = env_on("LAMM_HIP_GPU_QUANT") ? 1 : env_off("LAMM_HIP_GPU_QUANT") ? 0 : -1;
  k->fused = env_on("LAMM_HIP_FUSED");
  k->spin = !env_off("LAMM_HIP_SPIN");
  k->kernel_signal = env_on("LAMM_HIP_KERNEL_SIGNAL");
  k->c_watch = env_int("LAMM_HIP_C_WATCH", 0);
  k->direct = env_on("LAMM_HIP_DIRECT");
  k->aql_host_karg = env_on("LAMM_AQL_HOSTKARG");
  k->aql_eager = !env_off("LAMM_AQL_EAGER");
  {
    const char* f = getenv("LAMM_AQL_FENCE");
    k->aql_fence_none = f && !strcmp(f, "none");
  }
  k->vram_x = !env_off("LAMM_HIP_VRAM_X");
  k->signal_write = env_on("LAMM_HIP_SIGNAL_WRITE");
  k->siblings = !env_off("LAMM_HIP_SIBLINGS");
  const char* zc = getenv("LAMM_HIP_ZERO_COPY");
  k->zero_copy = !k->pinned || (zc && zc[0] == '0') ? 0 : zc && !strcmp(zc, "in") ? 1 : zc && !strcmp(zc, "out") ? 2 : 3;
  k->zero_copy_split = env_on("LAMM_HIP_ZERO_COPY_SPLIT");
  k->ref_mfma = env_int("LAMM_REF_MFMA", -1);
  k->ref_gemv_bpt = env_int("LAMM_REF_GEMV_BPT", 2);
  k->helpers = env_int("LAMM_HIP_HELPERS", 0);
  k->pool = env_int("LAMM_HIP_POOL", 5);
  if (const char* e = getenv("LAMM_HIP_ORDER")) k->ref_order = !strcmp(e, "reference") || !strcmp(e, "ref");
  return k;
}

std::atomic<const Knobs*> g_knobs{nullptr};

}  // namespace

const Knobs& knobs() {
  const Knobs* k = g_knobs.load(std::memory_order_acquire);
  if (k) return *k;
  const Knobs* fresh = read_env();
  if (!g_knobs.compare_exchange_strong(k, fresh, std::memory_order_acq_rel)) {
    delete fresh;   // another thread won; k holds its table
    return *k;
  }
  return *fresh;
}

// The previous table is leaked on purpose: a caller on another thread may still hold a reference.
void reload_knobs() { g_knobs.store(read_env(), std::memory_order_release); }

}  // namespace lamm

extern "C" void lamm_hip_reload_env(void) { lamm::reload_knobs(); }
