// engine_cells.hip -- alive counts, alive-cell lists and CellFlipped extraction, the per-turn flips
// ring.
//
// Reference roles: gol/distributor.go:153-166 (calculateAliveCells: an O(N^2) scan building the
// []util.Cell list, run every turn for the count), :53-59 (the per-turn diff that sends one
// CellFlipped per changed cell), :180-186 (TurnComplete).  Here the counts are fused into the
// stencil, and the lists come from a multi-block count / scan / emit over packed rows.
#include <algorithm>

#include "golhip_engine.hpp"

namespace golhip {

// Kernel variants whose launches can write a generation's flips beside their output (the
// production drift family; gol_step1 at K = 1).  The A/B-experiment variants cannot.
bool variant_writes_flips(int v) {
    return v == kVariantProd || v == kVariantDriftLds || v == kVariantDrift62 || v == kVariantPre63 ||
           v == kVariantProdMask;
}

// Extraction scratch for `rows` rows (a tall board of `slots` slots for the flips ring): grown,
// never shrunk -- a growth frees and reallocates, so it only happens for a larger ring.
int ensure_extract_scratch(golhip_t h, Shard &s, int64_t rows, int64_t slots) {
    if (rows <= s.ex_rows_cap && slots <= s.ex_slots_cap) return GOLHIP_OK;
    HIPCHK(h, hipSetDevice(s.device));
    SYNCCHK(h, s.compute);
    if (!s.ex_block_sums) HIPCHK(h, hipMalloc(&s.ex_block_sums, sizeof(unsigned long long) * kScanBlocks));
    if (rows > s.ex_rows_cap) {
        if (s.ex_rowcounts) HIPCHK(h, hipFree(s.ex_rowcounts));
        if (s.ex_offsets) HIPCHK(h, hipFree(s.ex_offsets));
        s.ex_rowcounts = nullptr;
        s.ex_offsets = nullptr;
        HIPCHK(h, hipMalloc(&s.ex_rowcounts, sizeof(uint32_t) * (size_t)rows));
        HIPCHK(h, hipMalloc(&s.ex_offsets, sizeof(unsigned long long) * (size_t)(rows + 1)));
        s.ex_rows_cap = rows;
    }
    if (slots > s.ex_slots_cap) {
        if (s.ex_slot_counts) HIPCHK(h, hipFree(s.ex_slot_counts));
        s.ex_slot_counts = nullptr;
        HIPCHK(h, hipMalloc(&s.ex_slot_counts, sizeof(unsigned long long) * (size_t)slots));
        s.ex_slots_cap = slots;
    }
    return GOLHIP_OK;
}

namespace {

// Cell lists, row-major (gol/distributor.go:153-166 alive cells, :53-59 flips): the set bits of
// a[i] (XOR b[i] when b is given) in the first `width` columns of each shard's rows.  slots > 1:
// a[i] is a tall board of `slots` consecutive boards of the shard's rows (the flips ring); the
// list is then slot-major (turn by turn), per_slot[t] = cells of slot t (nullable).  The scratch
// is preallocated; only a list longer than any before grows its output buffer.
int extract_cells(golhip_t h, const std::vector<const uint32_t *> &a, const std::vector<const uint32_t *> &b,
                  int64_t slots, int32_t *xy, size_t cap, size_t *n, uint64_t *per_slot) {
    if (!n) return fail(h, GOLHIP_ERR_ARG, "n is null");
    const size_t ns = h->shards.size();
    std::vector<std::vector<unsigned long long>> cnt(ns, std::vector<unsigned long long>(slots));
    for (size_t i = 0; i < ns; ++i) {
        Shard &s = h->shards[i];
        const int64_t rows = s.rows * slots;
        int rc = ensure_extract_scratch(h, s, rows, slots);
        if (rc) return rc;
        HIPCHK(h, hipSetDevice(s.device));
        HIPCHK(h, launch_extract_count(a[i], b[i], h->pitch, rows, h->width, s.ex_rowcounts, s.ex_offsets,
                                       s.ex_block_sums, s.compute));
        HIPCHK(h, launch_extract_slot_counts(s.ex_offsets, s.rows, slots, s.ex_slot_counts, s.compute));
        rc = copy_to_host(h, cnt[i].data(), s.ex_slot_counts, sizeof(unsigned long long) * (size_t)slots, s.compute);
        if (rc) return rc;
    }
    size_t total = 0;
    std::vector<size_t> shard_total(ns, 0);
    for (size_t i = 0; i < ns; ++i) {
        HIPCHK(h, hipSetDevice(h->shards[i].device));
        SYNCCHK(h, h->shards[i].compute);
        for (int64_t t = 0; t < slots; ++t) shard_total[i] += cnt[i][t];
        total += shard_total[i];
    }
    if (per_slot)
        for (int64_t t = 0; t < slots; ++t) {
            per_slot[t] = 0;
            for (size_t i = 0; i < ns; ++i) per_slot[t] += cnt[i][t];
        }
    *n = total;
    if (total > cap) return fail(h, GOLHIP_ERR_CAP, "%zu cells do not fit in cap %zu", total, cap);
    if (total == 0) return GOLHIP_OK;
    if (!xy) return fail(h, GOLHIP_ERR_ARG, "xy is null");
    // slot t of the output: the shards' cells of slot t in shard (row strip) order
    std::vector<size_t> slot_base(slots + 1, 0);
    for (int64_t t = 0; t < slots; ++t) {
        slot_base[t + 1] = slot_base[t];
        for (size_t i = 0; i < ns; ++i) slot_base[t + 1] += cnt[i][t];
    }
    for (size_t i = 0; i < ns; ++i) {
        Shard &s = h->shards[i];
        if (shard_total[i] == 0) continue;
        HIPCHK(h, hipSetDevice(s.device));
        if (shard_total[i] > s.ex_xy_cap) {  // grow the device list (rare: a longer list)
            SYNCCHK(h, s.compute);
            if (s.ex_xy) HIPCHK(h, hipFree(s.ex_xy));
            s.ex_xy = nullptr;
            const size_t want = std::max(shard_total[i], s.ex_xy_cap * 2);
            HIPCHK(h, hipMalloc(&s.ex_xy, sizeof(int32_t) * 2 * want));
            s.ex_xy_cap = want;
        }
        HIPCHK(h, launch_extract_emit(a[i], b[i], h->pitch, s.rows * slots, h->width, s.ex_offsets, s.y0,
                                      s.rows, s.ex_xy, shard_total[i], s.compute));
        // the shard's list is slot-major; copy each slot's run to its place in the global list
        // (one shard: the shard's list IS the global list, one copy)
        if (ns == 1) {
            HIPCHK(h, hipMemcpyAsync(xy, s.ex_xy, sizeof(int32_t) * 2 * shard_total[i], hipMemcpyDeviceToHost,
                                     s.compute));
            continue;
        }
        size_t src = 0;
        for (int64_t t = 0; t < slots; ++t) {
            size_t dst = slot_base[t];
            for (size_t i2 = 0; i2 < i; ++i2) dst += cnt[i2][t];
            if (cnt[i][t])
                HIPCHK(h, hipMemcpyAsync(xy + 2 * dst, s.ex_xy + 2 * src, sizeof(int32_t) * 2 * cnt[i][t],
                                         hipMemcpyDeviceToHost, s.compute));
            src += cnt[i][t];
        }
    }
    return sync_all(h);
}

// The flips ring as x-only rows (golhip_step_flips_rows / golhip_flips_fetch_rows): one strip
// per handle, width <= 65536.  row_offsets (slots * rows + 1 entries) = the exclusive scan of the
// ring's row counts, copied straight from the extraction scan; x = the cells' x as uint16 in the
// same order: 2 bytes per flip instead of the 8 of an (x, y) pair.
int extract_rows(golhip_t h, int64_t slots, uint16_t *x, size_t cap, size_t *n, uint64_t *row_offsets) {
    Shard &s = h->shards[0];
    const int64_t rows = s.rows * slots;
    int rc = ensure_extract_scratch(h, s, rows, slots);
    if (rc) return rc;
    HIPCHK(h, hipSetDevice(s.device));
    HIPCHK(h, launch_extract_count(s.ring, nullptr, h->pitch, rows, h->width, s.ex_rowcounts, s.ex_offsets,
                                   s.ex_block_sums, s.compute));
    rc = copy_to_host(h, row_offsets, s.ex_offsets, sizeof(uint64_t) * (size_t)(rows + 1), s.compute);
    if (rc) return rc;
    SYNCCHK(h, s.compute);
    const size_t total = (size_t)row_offsets[rows];
    *n = total;
    if (total > cap) return fail(h, GOLHIP_ERR_CAP, "%zu cells do not fit in cap %zu", total, cap);
    if (total == 0) return GOLHIP_OK;
    if (!x) return fail(h, GOLHIP_ERR_ARG, "x is null");
    if (total > s.ex_xy_cap) {  // the (x, y) list's device buffer holds 4x as many x-only cells
        if (s.ex_xy) HIPCHK(h, hipFree(s.ex_xy));
        s.ex_xy = nullptr;
        const size_t want = std::max(total, s.ex_xy_cap * 2);
        HIPCHK(h, hipMalloc(&s.ex_xy, sizeof(int32_t) * 2 * want));
        s.ex_xy_cap = want;
    }
    uint16_t *dx = reinterpret_cast<uint16_t *>(s.ex_xy);
    HIPCHK(h, launch_extract_emit_x16(s.ring, nullptr, h->pitch, rows, h->width, s.ex_offsets, dx, total,
                                      s.compute));
    HIPCHK(h, hipMemcpyAsync(x, dx, sizeof(uint16_t) * total, hipMemcpyDeviceToHost, s.compute));
    SYNCCHK(h, s.compute);
    return GOLHIP_OK;
}

// Ring slots per golhip_step_flips call: as many turns' flips boards as fit in ~1 GiB per strip
// (5120^2: 319 turns; 512^2: 1024; 65536^2: 2).  Every rank of a rank-mode board gets the same
// capacity (that of the largest strip, plan_rows), so a call that fits on one rank fits on all and
// no rank fails alone while the others block in the halo exchange.
int64_t ring_capacity(golhip_t h) {
    int64_t rows = std::max<int64_t>(1, plan_rows(h));
    for (auto &s : h->shards) rows = std::max(rows, s.rows);
    const int64_t board = rows * h->pitch * 4;
    return std::max<int64_t>(1, std::min<int64_t>(1024, ((int64_t)1 << 30) / board));
}

// The per-turn flips ring: allocated once per engine (ring_capacity turns of strip-sized slots).
int ensure_ring(golhip_t h, int64_t rc_cap) {
    if (h->ring_cap < rc_cap) {
        for (auto &s : h->shards) {
            HIPCHK(h, hipSetDevice(s.device));
            SYNCCHK(h, s.compute);
            if (s.ring) HIPCHK(h, hipFree(s.ring));
            s.ring = nullptr;
            HIPCHK(h, hipMalloc(&s.ring, sizeof(uint32_t) * (size_t)(rc_cap * s.rows * h->pitch)));
            int rc = ensure_extract_scratch(h, s, rc_cap * s.rows, rc_cap);
            if (rc) return rc;
        }
        h->ring_cap = rc_cap;
    }
    return GOLHIP_OK;
}

int rows_api_check(golhip_t h, uint64_t *row_offsets, size_t *n) {
    if (!h || !n || !row_offsets) return GOLHIP_ERR_ARG;
    if (h->shards.size() != 1)
        return fail(h, GOLHIP_ERR_STATE, "flips rows: one strip per handle (%zu here)", h->shards.size());
    if (h->width > 65536)
        return fail(h, GOLHIP_ERR_ARG, "flips rows: x is uint16, width %lld > 65536", (long long)h->width);
    return GOLHIP_OK;
}

}  // namespace
}  // namespace golhip

using namespace golhip;

// ================================================================================ C ABI ====
extern "C" {

int golhip_flips_ring_capacity(golhip_t h, int64_t *out) {
    if (!h || !out) return GOLHIP_ERR_ARG;
    *out = ring_capacity(h);
    return GOLHIP_OK;
}

int golhip_step_flips(golhip_t h, int64_t turns, int32_t *xy, size_t cap, size_t *n, uint64_t *flips_per_turn,
                      uint64_t *alive_per_turn) {
    if (!h || turns < 0 || !n) return GOLHIP_ERR_ARG;
    const int64_t rc_cap = ring_capacity(h);
    if (turns > rc_cap)
        return fail(h, GOLHIP_ERR_ARG, "%lld turns exceed the flips ring (%lld turns)", (long long)turns,
                    (long long)rc_cap);
    *n = 0;
    if (turns == 0) return GOLHIP_OK;
    int rc = ensure_ring(h, rc_cap);
    if (rc) return rc;
    rc = run_steps(h, turns, alive_per_turn, true);
    if (rc) return rc;
    h->ring_turns = turns;
    std::vector<const uint32_t *> a, b(h->shards.size(), nullptr);
    for (auto &s : h->shards) a.push_back(s.ring);
    return extract_cells(h, a, b, turns, xy, cap, n, flips_per_turn);
}

int golhip_flips_fetch(golhip_t h, int32_t *xy, size_t cap, size_t *n, uint64_t *flips_per_turn) {
    if (!h || !n) return GOLHIP_ERR_ARG;
    if (h->ring_turns == 0) return fail(h, GOLHIP_ERR_STATE, "no golhip_step_flips call holds flips in the ring");
    int rc = sync_all(h);
    if (rc) return rc;
    std::vector<const uint32_t *> a, b(h->shards.size(), nullptr);
    for (auto &s : h->shards) a.push_back(s.ring);
    return extract_cells(h, a, b, h->ring_turns, xy, cap, n, flips_per_turn);
}

int golhip_step_flips_rows(golhip_t h, int64_t turns, uint16_t *x, size_t cap, size_t *n, uint64_t *row_offsets,
                           uint64_t *alive_per_turn) {
    int rc = rows_api_check(h, row_offsets, n);
    if (rc) return rc;
    if (turns < 0) return GOLHIP_ERR_ARG;
    const int64_t rc_cap = ring_capacity(h);
    if (turns > rc_cap)
        return fail(h, GOLHIP_ERR_ARG, "%lld turns exceed the flips ring (%lld turns)", (long long)turns,
                    (long long)rc_cap);
    *n = 0;
    row_offsets[0] = 0;
    if (turns == 0) return GOLHIP_OK;
    rc = ensure_ring(h, rc_cap);
    if (rc) return rc;
    rc = run_steps(h, turns, alive_per_turn, true);
    if (rc) return rc;
    h->ring_turns = turns;
    return extract_rows(h, turns, x, cap, n, row_offsets);
}

int golhip_flips_fetch_rows(golhip_t h, uint16_t *x, size_t cap, size_t *n, uint64_t *row_offsets) {
    int rc = rows_api_check(h, row_offsets, n);
    if (rc) return rc;
    if (h->ring_turns == 0) return fail(h, GOLHIP_ERR_STATE, "no golhip_step_flips call holds flips in the ring");
    rc = sync_all(h);
    if (rc) return rc;
    return extract_rows(h, h->ring_turns, x, cap, n, row_offsets);
}

int golhip_track_flips(golhip_t h, int enable) {
    if (!h) return GOLHIP_ERR_ARG;
    if (enable && !variant_writes_flips(h->variant))
        return fail(h, GOLHIP_ERR_STATE, "flips need a production kernel variant (tuning variant %d cannot write them)",
                    h->variant);
    h->track_flips = enable != 0;
    if (h->track_flips)
        for (auto &s : h->shards)
            if (!s.diffbuf) {
                HIPCHK(h, hipSetDevice(s.device));
                HIPCHK(h, hipMalloc(&s.diffbuf, sizeof(uint32_t) * (size_t)(s.rows * h->pitch)));
            }
    return GOLHIP_OK;
}

int golhip_alive_count(golhip_t h, uint64_t *out) {
    if (!h || !out) return GOLHIP_ERR_ARG;
    std::vector<unsigned long long *> bufs;
    for (auto &s : h->shards) {
        HIPCHK(h, hipSetDevice(s.device));
        HIPCHK(h, hipMemsetAsync(s.scratch_u64, 0, sizeof(unsigned long long), s.compute));
        HIPCHK(h, launch_popcount(h->row0(s, h->cur), h->pitch, s.rows, h->wd, s.scratch_u64, s.compute));
        bufs.push_back(s.scratch_u64);
    }
    uint64_t v = 0;
    int rc = reduce_u64(h, bufs, 1, &v);
    if (rc) return rc;
    *out = v / (uint64_t)h->rep();
    return GOLHIP_OK;
}

int golhip_alive_cells(golhip_t h, int32_t *xy, size_t cap, size_t *n) {
    if (!h) return GOLHIP_ERR_ARG;
    int rc = sync_all(h);
    if (rc) return rc;
    std::vector<const uint32_t *> a, b(h->shards.size(), nullptr);
    for (auto &s : h->shards) a.push_back(h->row0(s, h->cur));
    return extract_cells(h, a, b, 1, xy, cap, n, nullptr);
}

int golhip_flips(golhip_t h, int32_t *xy, size_t cap, size_t *n) {
    if (!h) return GOLHIP_ERR_ARG;
    int rc = sync_all(h);
    if (rc) return rc;
    std::vector<const uint32_t *> a, b(h->shards.size(), nullptr);
    if (h->diff_valid) {  // written by the last launch beside its output
        for (auto &s : h->shards) a.push_back(s.diffbuf);
    } else if (h->prev_valid) {  // a one-generation launch: XOR with the buffer it read
        b.clear();
        for (auto &s : h->shards) {
            a.push_back(h->row0(s, h->cur));
            b.push_back(h->row0(s, h->cur ^ 1));
        }
    } else {
        if (n) *n = 0;
        return fail(h, GOLHIP_ERR_STATE,
                    "flips of the last generation are not held: enable golhip_track_flips (or step by 1 "
                    "turn) before stepping");
    }
    return extract_cells(h, a, b, 1, xy, cap, n, nullptr);
}

}  // extern "C"
