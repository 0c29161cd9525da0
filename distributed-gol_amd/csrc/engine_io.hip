// engine_io.hip -- the board in and out of the engine: PGM bytes, packed uint64 words, the random
// init regenerated on device, and checkpoint files.
//
// Reference roles: gol/io.go:42-128 (readPgmImage / writePgmImage: one channel op and one Write
// syscall per byte), broker/broker.go:124-155 + gol/distributor.go:69-91,139-147 (the broker's
// in-memory worldSave / turn that a later controller resumes: here a checkpoint file).
#include <algorithm>
#include <cstdio>
#include <cstring>

#include "golhip_engine.hpp"

namespace golhip {
namespace {

// Host <-> device byte transfer of the handle's rows, in row chunks through the shard's stage.
int transfer_bytes(golhip_t h, uint8_t *host, size_t row_stride, bool to_device) {
    if (!host) return fail(h, GOLHIP_ERR_ARG, "buffer is null");
    if (row_stride < (size_t)h->width) return fail(h, GOLHIP_ERR_ARG, "row_stride < width");
    const int64_t W = h->width;
    int64_t hrow = 0;  // host row index relative to the handle's first row
    for (auto &s : h->shards) {
        HIPCHK(h, hipSetDevice(s.device));
        uint8_t *stage = s.stage;
        const int64_t cr = std::min(std::max<int64_t>(1, s.stage_bytes / W), s.rows);
        for (int64_t y = 0; y < s.rows; y += cr) {
            const int64_t nr = std::min(cr, s.rows - y);
            uint32_t *rows_dev = h->row0(s, h->cur) + y * h->pitch;
            if (to_device) {
                HIPCHK(h, hipMemcpy2DAsync(stage, (size_t)W, host + (size_t)(hrow + y) * row_stride, row_stride,
                                           (size_t)W, (size_t)nr, hipMemcpyHostToDevice, s.compute));
                HIPCHK(h, launch_pack(stage, nr, W, h->wd, rows_dev, h->pitch, s.compute));
            } else {
                HIPCHK(h, launch_unpack(rows_dev, h->pitch, nr, W, stage, s.compute));
                HIPCHK(h, hipMemcpy2DAsync(host + (size_t)(hrow + y) * row_stride, row_stride, stage, (size_t)W,
                                           (size_t)W, (size_t)nr, hipMemcpyDeviceToHost, s.compute));
            }
            SYNCCHK(h, s.compute);
        }
        hrow += s.rows;
    }
    return GOLHIP_OK;
}

// ---- checkpoint (the broker's paused worldSave/turn/size, broker/broker.go:124-155) ----------
// File: a 64-byte little-endian header, then the handle's rows as packed bits, LSB-first
// (bit b of byte i of a row is x = 8i + b; the bits past `width` in a row's last byte are 0).
struct CkptHeader {
    char magic[8];  // "GOLCKPT1"
    uint32_t version, header_bytes;
    int64_t width, height, y0, rows, turn;
    uint64_t row_bytes;
};
static_assert(sizeof(CkptHeader) == 64, "checkpoint header layout");
const char kCkptMagic[8] = {'G', 'O', 'L', 'C', 'K', 'P', 'T', '1'};

int read_ckpt_header(FILE *f, CkptHeader *hd) {
    if (std::fread(hd, sizeof *hd, 1, f) != 1) return GOLHIP_ERR_ARG;
    if (std::memcmp(hd->magic, kCkptMagic, 8) != 0 || hd->version != 1 || hd->header_bytes != sizeof *hd ||
        hd->width <= 0 || hd->height <= 0 || hd->rows <= 0 || hd->row_bytes != (uint64_t)((hd->width + 7) / 8) ||
        hd->turn < 0)
        return GOLHIP_ERR_ARG;
    return GOLHIP_OK;
}

// Rows [y, y + nr) of a shard <-> packed host rows (row_bytes each).  Widths that are a multiple
// of 128 are the torus rows themselves (one 2-D copy); other widths go through the byte codec,
// which also restores the horizontal replication of the torus on load.
int ckpt_rows(golhip_t h, Shard &s, int64_t y, int64_t nr, uint8_t *host, bool to_device) {
    const int64_t W = h->width, rb = (W + 7) / 8;
    uint32_t *dev = h->row0(s, h->cur) + y * h->pitch;
    HIPCHK(h, hipSetDevice(s.device));
    if (W % 128 == 0) {
        if (to_device)
            HIPCHK(h, hipMemcpy2DAsync(dev, (size_t)h->pitch * 4, host, (size_t)rb, (size_t)rb, (size_t)nr,
                                       hipMemcpyHostToDevice, s.compute));
        else
            HIPCHK(h, hipMemcpy2DAsync(host, (size_t)rb, dev, (size_t)h->pitch * 4, (size_t)rb, (size_t)nr,
                                       hipMemcpyDeviceToHost, s.compute));
        SYNCCHK(h, s.compute);
        return GOLHIP_OK;
    }
    // the byte codec in row chunks through the shard's stage
    const int64_t cr = std::max<int64_t>(1, s.stage_bytes / W);
    std::vector<uint8_t> bytes((size_t)(std::min(cr, nr) * W));
    uint8_t *stage = s.stage;
    for (int64_t y0 = 0; y0 < nr; y0 += cr) {
        const int64_t n = std::min(cr, nr - y0);
        const size_t nb = (size_t)(n * W);
        uint8_t *hrows = host + y0 * rb;
        uint32_t *drows = dev + y0 * h->pitch;
        if (to_device) {
            for (int64_t r = 0; r < n; ++r)
                for (int64_t x = 0; x < W; ++x)
                    bytes[(size_t)(r * W + x)] = (hrows[r * rb + x / 8] >> (x % 8)) & 1 ? 255 : 0;
            HIPCHK(h, hipMemcpyAsync(stage, bytes.data(), nb, hipMemcpyHostToDevice, s.compute));
            HIPCHK(h, launch_pack(stage, n, W, h->wd, drows, h->pitch, s.compute));
            SYNCCHK(h, s.compute);
        } else {
            HIPCHK(h, launch_unpack(drows, h->pitch, n, W, stage, s.compute));
            HIPCHK(h, hipMemcpyAsync(bytes.data(), stage, nb, hipMemcpyDeviceToHost, s.compute));
            SYNCCHK(h, s.compute);
            std::memset(hrows, 0, (size_t)(n * rb));
            for (int64_t r = 0; r < n; ++r)
                for (int64_t x = 0; x < W; ++x)
                    if (bytes[(size_t)(r * W + x)]) hrows[r * rb + x / 8] |= (uint8_t)(1u << (x % 8));
        }
    }
    return GOLHIP_OK;
}

void board_replaced(golhip_t h) {
    h->turn = 0;
    h->prev_valid = false;
    h->diff_valid = false;
    h->act_valid = false;  // the stable-slab flags describe the old board
}

}  // namespace
}  // namespace golhip

using namespace golhip;

// ================================================================================ C ABI ====
extern "C" {

int golhip_load_bytes(golhip_t h, const uint8_t *cells, size_t row_stride) {
    if (!h) return GOLHIP_ERR_ARG;
    int rc = sync_all(h);
    if (rc) return rc;
    rc = transfer_bytes(h, const_cast<uint8_t *>(cells), row_stride, true);
    if (rc) return rc;
    board_replaced(h);
    return GOLHIP_OK;
}

int golhip_store_bytes(golhip_t h, uint8_t *out, size_t row_stride) {
    if (!h) return GOLHIP_ERR_ARG;
    int rc = sync_all(h);
    if (rc) return rc;
    return transfer_bytes(h, out, row_stride, false);
}

int golhip_init_random(golhip_t h, uint64_t seed, uint32_t density_q32) {
    if (!h) return GOLHIP_ERR_ARG;
    if (h->width % 64 != 0) return fail(h, GOLHIP_ERR_ARG, "init_random needs width %% 64 == 0");
    for (auto &s : h->shards) {
        HIPCHK(h, hipSetDevice(s.device));
        HIPCHK(h, launch_init_random(h->row0(s, h->cur), h->pitch, s.rows, s.y0, h->width, h->wd, seed, density_q32,
                                     s.compute));
    }
    board_replaced(h);
    return sync_all(h);
}

int golhip_store_words(golhip_t h, uint64_t *out) {
    if (!h || !out) return GOLHIP_ERR_ARG;
    if (h->width % 64 != 0) return fail(h, GOLHIP_ERR_ARG, "store_words needs width %% 64 == 0");
    int rc = sync_all(h);
    if (rc) return rc;
    const int64_t wpr = h->width / 64;
    int64_t hrow = 0;
    for (auto &s : h->shards) {
        HIPCHK(h, hipSetDevice(s.device));
        uint64_t *d = reinterpret_cast<uint64_t *>(s.stage);
        const int64_t cr = std::max<int64_t>(1, s.stage_bytes / (int64_t)sizeof(uint64_t) / wpr);
        for (int64_t y = 0; y < s.rows; y += cr) {
            const int64_t nr = std::min(cr, s.rows - y);
            HIPCHK(h, launch_words_out(h->row0(s, h->cur) + y * h->pitch, h->pitch, nr, h->width, d, s.compute));
            HIPCHK(h, hipMemcpyAsync(out + (hrow + y) * wpr, d, sizeof(uint64_t) * (size_t)(nr * wpr),
                                     hipMemcpyDeviceToHost, s.compute));
            SYNCCHK(h, s.compute);
        }
        hrow += s.rows;
    }
    return GOLHIP_OK;
}

int golhip_load_words(golhip_t h, const uint64_t *in) {
    if (!h || !in) return GOLHIP_ERR_ARG;
    if (h->width % 64 != 0) return fail(h, GOLHIP_ERR_ARG, "load_words needs width %% 64 == 0");
    int rc = sync_all(h);
    if (rc) return rc;
    const int64_t wpr = h->width / 64;
    int64_t hrow = 0;
    for (auto &s : h->shards) {
        HIPCHK(h, hipSetDevice(s.device));
        uint64_t *d = reinterpret_cast<uint64_t *>(s.stage);
        const int64_t cr = std::max<int64_t>(1, s.stage_bytes / (int64_t)sizeof(uint64_t) / wpr);
        for (int64_t y = 0; y < s.rows; y += cr) {
            const int64_t nr = std::min(cr, s.rows - y);
            HIPCHK(h, hipMemcpyAsync(d, in + (hrow + y) * wpr, sizeof(uint64_t) * (size_t)(nr * wpr),
                                     hipMemcpyHostToDevice, s.compute));
            HIPCHK(h, launch_words_in(d, nr, h->width, h->wd, h->row0(s, h->cur) + y * h->pitch, h->pitch,
                                      s.compute));
            SYNCCHK(h, s.compute);
        }
        hrow += s.rows;
    }
    board_replaced(h);
    return GOLHIP_OK;
}

int golhip_checkpoint_info(const char *path, int64_t *width, int64_t *height, int64_t *turn) {
    if (!path) return GOLHIP_ERR_ARG;
    FILE *f = std::fopen(path, "rb");
    if (!f) return GOLHIP_ERR_ARG;
    CkptHeader hd;
    const int rc = read_ckpt_header(f, &hd);
    std::fclose(f);
    if (rc) return rc;
    if (width) *width = hd.width;
    if (height) *height = hd.height;
    if (turn) *turn = hd.turn;
    return GOLHIP_OK;
}

int golhip_checkpoint_save(golhip_t h, const char *path) {
    if (!h || !path) return GOLHIP_ERR_ARG;
    int rc = sync_all(h);
    if (rc) return rc;
    const std::string tmp = std::string(path) + ".tmp";
    FILE *f = std::fopen(tmp.c_str(), "wb");
    if (!f) return fail(h, GOLHIP_ERR_ARG, "cannot write %s", tmp.c_str());
    CkptHeader hd{};
    std::memcpy(hd.magic, kCkptMagic, 8);
    hd.version = 1;
    hd.header_bytes = sizeof hd;
    hd.width = h->width;
    hd.height = h->height;
    hd.y0 = h->shards.front().y0;
    hd.rows = 0;
    for (auto &s : h->shards) hd.rows += s.rows;
    hd.turn = h->turn;
    hd.row_bytes = (uint64_t)((h->width + 7) / 8);
    bool ok = std::fwrite(&hd, sizeof hd, 1, f) == 1;
    const int64_t chunk = std::max<int64_t>(1, (64ll << 20) / (int64_t)hd.row_bytes);
    std::vector<uint8_t> buf;
    for (auto &s : h->shards)
        for (int64_t y = 0; ok && y < s.rows; y += chunk) {
            const int64_t nr = std::min(chunk, s.rows - y);
            buf.resize((size_t)(nr * (int64_t)hd.row_bytes));
            if ((rc = ckpt_rows(h, s, y, nr, buf.data(), false))) break;
            ok = std::fwrite(buf.data(), 1, buf.size(), f) == buf.size();
        }
    ok = (std::fclose(f) == 0) && ok;
    if (rc || !ok) {
        std::remove(tmp.c_str());
        return rc ? rc : fail(h, GOLHIP_ERR_ARG, "short write to %s", tmp.c_str());
    }
    if (std::rename(tmp.c_str(), path) != 0) {  // atomic replace: never a half-written checkpoint
        std::remove(tmp.c_str());
        return fail(h, GOLHIP_ERR_ARG, "cannot rename %s to %s", tmp.c_str(), path);
    }
    return GOLHIP_OK;
}

int golhip_checkpoint_load(golhip_t h, const char *path) {
    if (!h || !path) return GOLHIP_ERR_ARG;
    int rc = sync_all(h);
    if (rc) return rc;
    FILE *f = std::fopen(path, "rb");
    if (!f) return fail(h, GOLHIP_ERR_ARG, "cannot read %s", path);
    CkptHeader hd;
    if ((rc = read_ckpt_header(f, &hd))) {
        std::fclose(f);
        return fail(h, rc, "%s is not a golhip checkpoint", path);
    }
    int64_t rows = 0;
    for (auto &s : h->shards) rows += s.rows;
    if (hd.width != h->width || hd.height != h->height || hd.y0 != h->shards.front().y0 || hd.rows != rows) {
        std::fclose(f);
        return fail(h, GOLHIP_ERR_STATE,
                    "checkpoint holds rows [%lld, %lld) of a %lldx%lld board, this handle rows [%lld, %lld) "
                    "of %lldx%lld",
                    (long long)hd.y0, (long long)(hd.y0 + hd.rows), (long long)hd.width, (long long)hd.height,
                    (long long)h->shards.front().y0, (long long)(h->shards.front().y0 + rows),
                    (long long)h->width, (long long)h->height);
    }
    const int64_t chunk = std::max<int64_t>(1, (64ll << 20) / (int64_t)hd.row_bytes);
    std::vector<uint8_t> buf;
    bool ok = true;
    for (auto &s : h->shards)
        for (int64_t y = 0; ok && y < s.rows; y += chunk) {
            const int64_t nr = std::min(chunk, s.rows - y);
            buf.resize((size_t)(nr * (int64_t)hd.row_bytes));
            ok = std::fread(buf.data(), 1, buf.size(), f) == buf.size();
            if (ok && (rc = ckpt_rows(h, s, y, nr, buf.data(), true))) break;
        }
    std::fclose(f);
    if (rc) return rc;
    if (!ok) return fail(h, GOLHIP_ERR_ARG, "%s is truncated", path);
    h->turn = hd.turn;
    h->prev_valid = false;
    h->diff_valid = false;
    h->act_valid = false;
    return GOLHIP_OK;
}

}  // extern "C"
