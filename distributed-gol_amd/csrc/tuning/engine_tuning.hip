// tuning/engine_tuning.hip -- tuning library only: the engine hooks (golhip_engine.hpp EngineHooks)
// of the A/B experiments and the fault-injection tests.  The production library does not contain
// this TU, so none of these environment variables reaches it.
//
//   A/B selectors, read at create (scripts/ab_*.py, scripts/tune_*.py, tests/test_gpu_tuning.py):
//     GOLHIP_VARIANT        stencil variant (golhip_internal.hpp kVariant*; "prod" = production)
//     GOLHIP_SPLIT / GOLHIP_TILE / GOLHIP_SLAB   force the level split / register tile / slab shape
//     GOLHIP_BAND_ROWS, GOLHIP_FIXED_K, GOLHIP_COUNT_WINDOW, GOLHIP_GRAPHS
//     GOLHIP_EDGE_PRIO / GOLHIP_EDGE_FIRST / GOLHIP_EDGE_SETPRIO   the split step's streams
//     GOLHIP_LDS_PAD        unused dynamic LDS per stencil block (read when the library loads)
//   Fault injection (tests/test_gpu_failfast.py):
//     GOLHIP_FAULT=stall      every golhip_step ends in a 20 s stall of the compute stream (a rank
//                             whose device work does not finish; nothing RCCL queued behind it)
//     GOLHIP_FAULT=skip_send  the first send of every halo exchange from exchange number
//                             GOLHIP_FAULT_FROM (default 1) on is left out of the RCCL group: the
//                             peer's matching receive never completes (a stuck RCCL transfer)
//     GOLHIP_FAULT=slab_stall golhip_step_persistent's slab 0 never signals its first block: its
//                             neighbours time out (a slab that is not resident)
//   Timestamps: GOLHIP_VARIANT=stamp -- per-wave stamps of the last single-strip launch
//     (golhip_tuning_stamps / golhip_tuning_stamps_ex; scripts/stamp_launch.py, slab_stamps.py).
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "../golhip_engine.hpp"

namespace golhip {
namespace {

int env_int(const char *name, int dflt) {
    const char *e = std::getenv(name);
    return e ? std::atoi(e) : dflt;
}

void configure(golhip_t h) {
    if (const char *e = std::getenv("GOLHIP_BAND_ROWS")) h->band_rows = std::atoi(e);
    // measurement knob (scripts/pmc_passes.sh): every bulk launch exactly k deep, as
    // golhip_set_fixed_k(h, 1) -- the planner would otherwise run its fastest depth <= k
    if (const char *e = std::getenv("GOLHIP_FIXED_K")) h->fixed_k = std::atoi(e) != 0;
    if (const char *e = std::getenv("GOLHIP_COUNT_WINDOW")) h->count_window = std::max(kCountWindowMin, std::atoi(e));
    if (const char *e = std::getenv("GOLHIP_GRAPHS")) h->graph_mode = std::atoi(e) != 0;
    h->force_split = env_int("GOLHIP_SPLIT", h->force_split);
    h->force_tile = env_int("GOLHIP_TILE", h->force_tile);
    h->force_slab = env_int("GOLHIP_SLAB", h->force_slab);
    h->edge_prio = env_int("GOLHIP_EDGE_PRIO", 0) != 0;
    h->edge_first = env_int("GOLHIP_EDGE_FIRST", 0) != 0;
    h->edge_setprio = env_int("GOLHIP_EDGE_SETPRIO", 1) != 0;
    if (const char *e = std::getenv("GOLHIP_VARIANT")) {
        static const struct {
            const char *name;
            int v;
        } kNames[] = {{"chain", kVariantChain},         {"skew", kVariantSkew},
                      {"skew2", kVariantSkewD2},        {"chain2", kVariantChainD2},
                      {"skewlds", kVariantSkewLdsPf},   {"skewlds2", kVariantSkewLdsD2},
                      {"chainlds2", kVariantChainLdsD2}, {"chainlds", kVariantChainLdsPf},
                      {"driftzip", kVariantDriftZip},   {"drift62", kVariantDrift62},
                      {"driftnf", kVariantDriftNoFill}, {"driftlds", kVariantDriftLds},
                      {"pre63", kVariantPre63},         {"prodmask", kVariantProdMask},
                      {"stamp", kVariantStamp}};
        h->variant = kVariantProd;
        for (const auto &n : kNames)
            if (std::strcmp(e, n.name) == 0) h->variant = n.v;
    }
    if (const char *e = std::getenv("GOLHIP_FAULT")) {
        if (std::strcmp(e, "stall") == 0) h->fault = Fault::stall;
        if (std::strcmp(e, "skip_send") == 0) h->fault = Fault::skip_send;
        if (std::strcmp(e, "slab_stall") == 0) h->fault = Fault::slab_stall;
    }
}

int create(golhip_t h) {
    if (h->variant != kVariantStamp) return GOLHIP_OK;
    HIPCHK(h, hipSetDevice(h->shards[0].device));
    HIPCHK(h, hipMalloc(&h->stamp_buf, sizeof(uint64_t) * 4 * kStampWaves));
    return GOLHIP_OK;
}

void destroy(golhip_t h) {
    if (h->stamp_buf) (void)hipFree(h->stamp_buf);
    h->stamp_buf = nullptr;
}

// The stamp variant's streaming gol_stencil writes p.diff as its stamps.  ONLY that kernel:
// gol_step1 (K = 1) and the register kernels read a non-null p.diff as a flips board of the strip's
// size (round 4: a K = 1 warmup launch wrote its flips over the 32 MiB stamp buffer -- an illegal
// memory access, profiles/r04/r04d_stamps_fault.log; tests/test_gpu_tuning.py
// test_stamp_variant_k1_then_deep pins this).  gol_slab2 / gol_slab3 write their phase stamps
// through p.stamp.
void launch_params(golhip_t h, const Shard &s, int K, bool counting, StencilParams &p) {
    if (!h->stamp_buf || p.diff || K <= 1) return;
    const RegKernel rk = pick_reg_kernel(h, s.rows, K, counting);
    if (rk.kind == 0 && pick_split(h, s.rows, K) <= 1 && p.nbands * (int64_t)p.nchunks <= kStampWaves) {
        p.diff = reinterpret_cast<uint32_t *>(h->stamp_buf);
        h->stamp_waves = p.nbands * (int64_t)p.nchunks;
        h->stamp_words = 4;
    } else if (rk.kind == 3 && rk.NC >= 9 && rk.NC <= 13 &&
               8 * p.nbands * (int64_t)p.nchunks * rk.W <= 4 * kStampWaves) {
        p.stamp = h->stamp_buf;
        h->stamp_waves = p.nbands * (int64_t)p.nchunks * rk.W;
        h->stamp_words = 8;
    }
}

int after_steps(golhip_t h) {
    if (h->fault != Fault::stall || !rccl_waits(h)) return GOLHIP_OK;
    HIPCHK(h, hipLaunchHostFunc(h->shards[0].compute,
                                [](void *) { std::this_thread::sleep_for(std::chrono::seconds(20)); }, nullptr));
    return GOLHIP_OK;
}

bool skip_xfer(golhip_t h, const golhip_xfer &x, int i) {
    static const int from = env_int("GOLHIP_FAULT_FROM", 1);
    return h->fault == Fault::skip_send && x.kind == 0 && i == 0 && h->exchanges >= from;
}

const EngineHooks kHooks = [] {
    EngineHooks k;
    k.configure = configure;
    k.create = create;
    k.destroy = destroy;
    k.launch_params = launch_params;
    k.after_steps = after_steps;
    k.skip_xfer = skip_xfer;
    return k;
}();

const bool registered = [] {
    set_engine_hooks(&kHooks);
    if (const char *e = std::getenv("GOLHIP_LDS_PAD")) kernel_extras().lds_pad = (size_t)std::atol(e);
    return true;
}();

}  // namespace
}  // namespace golhip

using namespace golhip;

extern "C" {

// Tuning library only (not in include/golhip.h): the per-wave stamps of the last single-strip
// launch of a GOLHIP_VARIANT=stamp handle, 4 uint64 per wave (start, end: s_memrealtime 100 MHz;
// shader cycles; HW_ID | XCC_ID << 32).  scripts/stamp_launch.py.
int golhip_tuning_stamps(golhip_t h, uint64_t *out, size_t cap_waves, size_t *n_waves) {
    if (!h || !n_waves) return GOLHIP_ERR_ARG;
    if (!h->stamp_buf) return fail(h, GOLHIP_ERR_STATE, "not a GOLHIP_VARIANT=stamp handle");
    int rc = sync_all(h);
    if (rc) return rc;
    *n_waves = (size_t)std::min<int64_t>(h->stamp_waves, kStampWaves);
    if (!out) return GOLHIP_OK;
    if (cap_waves < *n_waves) return GOLHIP_ERR_CAP;
    HIPCHK(h, hipMemcpy(out, h->stamp_buf, sizeof(uint64_t) * 4 * *n_waves, hipMemcpyDeviceToHost));
    return GOLHIP_OK;
}

// The same with the record length: words_per_wave uint64 per wave (4: gol_stencil, 8: gol_slab2's
// phase stamps -- start, rows loaded, generations done, end, cycles, HW_ID | XCC_ID << 32, group,
// wave).  cap_words / n_words count uint64.  scripts/slab_stamps.py.
int golhip_tuning_stamps_ex(golhip_t h, uint64_t *out, size_t cap_words, size_t *n_words, int *words_per_wave) {
    if (!h || !n_words || !words_per_wave) return GOLHIP_ERR_ARG;
    if (!h->stamp_buf) return fail(h, GOLHIP_ERR_STATE, "not a GOLHIP_VARIANT=stamp handle");
    int rc = sync_all(h);
    if (rc) return rc;
    *words_per_wave = h->stamp_words;
    *n_words = (size_t)std::min<int64_t>(h->stamp_waves * h->stamp_words, 4 * kStampWaves);
    if (!out) return GOLHIP_OK;
    if (cap_words < *n_words) return GOLHIP_ERR_CAP;
    HIPCHK(h, hipMemcpy(out, h->stamp_buf, sizeof(uint64_t) * *n_words, hipMemcpyDeviceToHost));
    return GOLHIP_OK;
}

}  // extern "C"
