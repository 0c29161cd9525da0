/*
 * gol_oracle.c -- CPU ORACLE for the Game-of-Life hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / the timed CPU baseline.  The product path
 * (distributed-gol_amd/, libgolhip) never links, loads or calls anything here.
 *
 * Two restatements live here:
 *
 *  1. oracle_ref_*  -- a line-by-line *behavioural* restatement of the reference's
 *     byte-per-cell compute path (Oliver-Cairns/distributed-gol, pure Go):
 *       - countAliveCellsAdjacent   server/server.go:55-75   (torus wrap by 4 branches, sum/255)
 *       - updateCell                server/server.go:33-53   (B3/S23 ladder on 0/255 bytes)
 *       - calculateNextState        server/server.go:21-31   (fresh row allocation per turn)
 *       - GolOP.Work thread split   server/server.go:83-104  (SplitSize/Threads, remainder first)
 *       - broker publish split      broker/broker.go:37-56   (ImageSize/numServers strips)
 *       - Broker.Publish stitch     broker/broker.go:157-180 (ordered concatenation)
 *     It keeps the reference's cost structure (bytes, branches, per-turn row allocation,
 *     servers x threads workers -- a persistent pool, the goroutine analogue -- and an optional
 *     full-world copy per server per turn modelling the gob fan-out of broker/broker.go:51) and
 *     is the `cpu_baseline` "port".
 *
 *  2. oracle_packed_* -- an independent bit-sliced stepper (64 cells per uint64, LSB-first:
 *     bit b of word j is x = 64j+b) used to produce golden vectors at sizes the byte
 *     restatement cannot reach in seconds.  It is pinned against (1) and against the
 *     reference's own fixtures (tests/golden/reference/check/...) by tests/test_oracle.py.
 *
 * Parity is PINNED: (1) and (2) reproduce all 9 check/images PGMs byte-exact and all
 * 30000 counts of the check/alive CSVs (tests/test_oracle.py).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------ */
/* 1. Reference-algorithm restatement (byte per cell, 0 = dead, 255 = alive)            */
/* ------------------------------------------------------------------------------------ */

/* server/server.go:55-75 */
static int ref_count_adjacent(int height, int width, uint8_t **world, int x, int y) {
    int left = x - 1, right = x + 1, up = y - 1, down = y + 1;
    int count = 0;
    if (x == 0) left = width - 1;
    if (x == width - 1) right = 0;
    if (y == 0) up = height - 1;
    if (y == height - 1) down = 0;
    count += (int)world[up][left] + (int)world[up][x] + (int)world[up][right] +
             (int)world[y][left] + (int)world[y][right] +
             (int)world[down][left] + (int)world[down][x] + (int)world[down][right];
    count /= 255;
    return count;
}

/* server/server.go:33-53 */
static uint8_t ref_update_cell(int height, int width, uint8_t **world, int x, int y) {
    int alive = ref_count_adjacent(height, width, world, x, y);
    if (world[y][x] == 0) {
        if (alive == 3) return 255;
        return 0;
    }
    if (world[y][x] == 255) {
        if (alive < 2) return 0;
        if (alive == 2 || alive == 3) return 255;
        if (alive > 3) return 0;
    }
    return 1;
}

typedef struct {
    int image_size, start, end;
    uint8_t **world;
    uint8_t **rows_out; /* filled with end-start+1 freshly malloc'd rows */
} ref_task;

/* server/server.go:21-31 -- one goroutine's sub-strip, fresh rows every turn */
static void *ref_calculate_next_state(void *arg) {
    ref_task *t = (ref_task *)arg;
    int split_height = t->end - t->start + 1;
    for (int y = 0; y < split_height; y++) {
        uint8_t *row = (uint8_t *)malloc((size_t)t->image_size);
        for (int x = 0; x < t->image_size; x++)
            row[x] = ref_update_cell(t->image_size, t->image_size, t->world, x, y + t->start);
        t->rows_out[y] = row;
    }
    return NULL;
}

/*
 * The reference's workers, as a persistent pool (the goroutine analogue): servers x threads
 * workers are created ONCE per run and handed each turn's work through barriers, so a turn costs
 * what a Go turn costs -- spawning goroutines is cheap, spawning OS threads per turn is not
 * (round 3 created 256 pthreads per turn, which dominated the 512^2 figure).  Per turn:
 *   1. fan-out: the first worker of each server copies the whole world (the server's gob-decoded
 *      private copy, broker/broker.go:51,64; the servers are separate processes, so the copies run
 *      concurrently), when fanout_copy != 0;
 *   2. every worker computes its sub-strip into freshly malloc'd rows (server/server.go:21-31,
 *      83-97: SplitSize/Threads rows, remainder first);
 *   3. the calling thread stitches the rows in server then goroutine order (broker/broker.go:168-174,
 *      server/server.go:98-104) and frees them.
 */
typedef struct ref_pool ref_pool;
typedef struct {
    ref_pool *pool;
    int server, index;
} ref_worker;

struct ref_pool {
    int n, servers, threads, fanout;
    int nw;                       /* servers * threads */
    const uint8_t *world;         /* this turn's input */
    uint8_t **rows;               /* Request.World as [][]byte: row slices into `world` */
    uint8_t **server_block;       /* fan-out copies, n*n bytes per server */
    uint8_t ***server_world;      /* row slices into them */
    ref_task *tasks;              /* nw sub-strips (fixed split) */
    ref_worker *workers;
    pthread_t *tids;
    pthread_barrier_t start, copied, done;
    int quit;
};

static void *ref_worker_main(void *arg) {
    ref_worker *w = (ref_worker *)arg;
    ref_pool *p = w->pool;
    for (;;) {
        pthread_barrier_wait(&p->start);
        if (p->quit) break;
        if (p->fanout && w->index == 0)
            memcpy(p->server_block[w->server], p->world, (size_t)p->n * p->n);
        pthread_barrier_wait(&p->copied);
        ref_calculate_next_state(&p->tasks[w->server * p->threads + w->index]);
        pthread_barrier_wait(&p->done);
    }
    return NULL;
}

static void ref_pool_destroy(ref_pool *p) {
    if (!p) return;
    if (p->tids) {
        p->quit = 1;
        pthread_barrier_wait(&p->start);
        for (int i = 0; i < p->nw; i++) pthread_join(p->tids[i], NULL);
        pthread_barrier_destroy(&p->start);
        pthread_barrier_destroy(&p->copied);
        pthread_barrier_destroy(&p->done);
    }
    for (int s = 0; p->server_block && s < p->servers; s++) {
        free(p->server_world[s]);
        free(p->server_block[s]);
    }
    for (int i = 0; p->tasks && i < p->nw; i++) free(p->tasks[i].rows_out);
    free(p->server_world);
    free(p->server_block);
    free(p->tasks);
    free(p->workers);
    free(p->tids);
    free(p->rows);
    free(p);
}

/* n % servers != 0 is rejected: the reference's own index arithmetic drops rows there
 * (SURVEY.md section 0 fact 5). */
static ref_pool *ref_pool_create(int n, int threads, int servers, int fanout_copy) {
    if (n <= 0 || threads <= 0 || servers <= 0 || n % servers != 0) return NULL;
    ref_pool *p = (ref_pool *)calloc(1, sizeof(ref_pool));
    p->n = n;
    p->servers = servers;
    p->threads = threads;
    p->fanout = fanout_copy;
    p->nw = servers * threads;
    p->rows = (uint8_t **)malloc(sizeof(uint8_t *) * (size_t)n);
    p->tasks = (ref_task *)calloc((size_t)p->nw, sizeof(ref_task));
    p->workers = (ref_worker *)calloc((size_t)p->nw, sizeof(ref_worker));
    p->server_block = (uint8_t **)calloc((size_t)servers, sizeof(uint8_t *));
    p->server_world = (uint8_t ***)calloc((size_t)servers, sizeof(uint8_t **));
    if (fanout_copy)
        for (int s = 0; s < servers; s++) {
            p->server_block[s] = (uint8_t *)malloc((size_t)n * n);
            p->server_world[s] = (uint8_t **)malloc(sizeof(uint8_t *) * (size_t)n);
            if (!p->server_block[s] || !p->server_world[s]) {
                ref_pool_destroy(p);
                return NULL;
            }
            for (int y = 0; y < n; y++) p->server_world[s][y] = p->server_block[s] + (size_t)y * n;
        }
    /* broker publish: splitSize := ImageSize / numServers (broker/broker.go:38-51);
     * GolOP.Work: splitSize := req.SplitSize / req.Threads (server/server.go:83-97) */
    int split = n / servers, diff = n % servers, pos = 0;
    for (int s = 0; s < servers; s++) {
        int start = pos;
        pos += split - 1;
        if (diff != 0) { pos++; diff--; }
        pos++;
        int tsplit = split / threads, tdiff = split % threads, tpos = start;
        for (int i = 0; i < threads; i++) {
            int tstart = tpos;
            tpos += tsplit - 1;
            if (tdiff > 0) { tpos++; tdiff--; }
            int tend = tpos;
            tpos++;
            ref_task *t = &p->tasks[s * threads + i];
            t->image_size = n;
            t->start = tstart;
            t->end = tend;
            t->world = fanout_copy ? p->server_world[s] : p->rows;
            int h = tend - tstart + 1;
            t->rows_out = (uint8_t **)malloc(sizeof(uint8_t *) * (size_t)(h > 0 ? h : 1));
        }
    }
    pthread_barrier_init(&p->start, NULL, (unsigned)p->nw + 1);
    pthread_barrier_init(&p->copied, NULL, (unsigned)p->nw);
    pthread_barrier_init(&p->done, NULL, (unsigned)p->nw + 1);
    p->tids = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)p->nw);
    for (int s = 0; s < servers; s++)
        for (int i = 0; i < threads; i++) {
            ref_worker *w = &p->workers[s * threads + i];
            w->pool = p;
            w->server = s;
            w->index = i;
            pthread_create(&p->tids[s * threads + i], NULL, ref_worker_main, w);
        }
    return p;
}

/* One turn through the pool: world -> out (n*n bytes each).  Returns the rows produced. */
static int ref_pool_step(ref_pool *p, const uint8_t *world, uint8_t *out) {
    const int n = p->n;
    p->world = world;
    for (int y = 0; y < n; y++) p->rows[y] = (uint8_t *)world + (size_t)y * n;
    pthread_barrier_wait(&p->start);
    pthread_barrier_wait(&p->done);
    int produced = 0;
    for (int i = 0; i < p->nw; i++) {
        int h = p->tasks[i].end - p->tasks[i].start + 1;
        for (int y = 0; y < h; y++) {
            if (produced < n) memcpy(out + (size_t)produced * n, p->tasks[i].rows_out[y], (size_t)n);
            produced++;
            free(p->tasks[i].rows_out[y]);
        }
    }
    return produced;
}

/*
 * One reference turn: broker fan-out to `servers` strips (broker/broker.go:37-56), each
 * server splitting req.SplitSize rows over `threads` goroutines (server/server.go:83-97),
 * strips stitched in order (broker/broker.go:168-174, server/server.go:98-104).
 *
 * world/out: n*n bytes, row-major.  Returns the number of rows produced (== n for the
 * reference-supported case n % servers == 0), or -1 when the reference's own index
 * arithmetic would drop rows (n % servers != 0).
 * If fanout_copy != 0, each server first receives a private copy of the whole world,
 * modelling the per-server gob encode of the full board (broker/broker.go:51,64).
 */
int oracle_ref_step(int n, const uint8_t *world, uint8_t *out, int threads, int servers,
                    int fanout_copy) {
    ref_pool *p = ref_pool_create(n, threads, servers, fanout_copy);
    if (!p) return -1;
    int produced = ref_pool_step(p, world, out);
    ref_pool_destroy(p);
    return produced;
}

/* Run `turns` reference turns in place (world n*n bytes) on one worker pool.  counts (nullable,
 * len turns) receives the alive count after each completed turn, as gol/distributor.go:153-166,186
 * (the controller's scan, one thread). */
int oracle_ref_run(int n, uint8_t *world, long turns, int threads, int servers, int fanout_copy,
                   int64_t *counts) {
    ref_pool *p = ref_pool_create(n, threads, servers, fanout_copy);
    if (!p) return -1;
    uint8_t *tmp = (uint8_t *)malloc((size_t)n * n);
    for (long t = 0; t < turns; t++) {
        int r = ref_pool_step(p, world, tmp);
        if (r != n) { free(tmp); ref_pool_destroy(p); return -1; }
        memcpy(world, tmp, (size_t)n * n);
        if (counts) {
            int64_t c = 0;
            for (size_t i = 0; i < (size_t)n * n; i++) c += world[i] == 255;
            counts[t] = c;
        }
    }
    free(tmp);
    ref_pool_destroy(p);
    return 0;
}

/* ------------------------------------------------------------------------------------ */
/* 2. Bit-packed stepper (independent algorithm, pinned against 1. and the fixtures)    */
/* ------------------------------------------------------------------------------------ */

/* B3/S23 on 64 cells: a/b/d = rows above/own/below, *l / *r = the words to the west/east. */
static inline uint64_t life64(uint64_t al, uint64_t a, uint64_t ar, uint64_t bl, uint64_t b,
                              uint64_t br, uint64_t dl, uint64_t d, uint64_t dr) {
    /* west neighbour (x-1) moved onto x, east neighbour (x+1) moved onto x */
    uint64_t aw = (a << 1) | (al >> 63), ae = (a >> 1) | (ar << 63);
    uint64_t bw = (b << 1) | (bl >> 63), be = (b >> 1) | (br << 63);
    uint64_t dw = (d << 1) | (dl >> 63), de = (d >> 1) | (dr << 63);
    /* plain per-bit 8-neighbour count as 4 bit-planes s0..s3 (ripple counter) */
    uint64_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
#define ORACLE_ADD(v)                                   \
    do {                                                \
        uint64_t c0 = s0 & (v); s0 ^= (v);              \
        uint64_t c1 = s1 & c0; s1 ^= c0;                \
        uint64_t c2 = s2 & c1; s2 ^= c1;                \
        s3 ^= c2;                                       \
    } while (0)
    ORACLE_ADD(aw); ORACLE_ADD(a); ORACLE_ADD(ae); ORACLE_ADD(bw);
    ORACLE_ADD(be); ORACLE_ADD(dw); ORACLE_ADD(d); ORACLE_ADD(de);
#undef ORACLE_ADD
    uint64_t is3 = s0 & s1 & ~s2 & ~s3, is2 = ~s0 & s1 & ~s2 & ~s3;
    return is3 | (is2 & b);
}

/* One generation of rows [y0, y1) of a wpr-words-per-row torus of height h. */
static void packed_rows(int wpr, int h, const uint64_t *in, uint64_t *out, int y0, int y1,
                        int64_t *count) {
    int64_t c = 0;
    for (int y = y0; y < y1; y++) {
        const uint64_t *ra = in + (size_t)((y + h - 1) % h) * wpr;
        const uint64_t *rb = in + (size_t)y * wpr;
        const uint64_t *rc = in + (size_t)((y + 1) % h) * wpr;
        uint64_t *ro = out + (size_t)y * wpr;
        if (wpr == 1) {
            ro[0] = life64(ra[0], ra[0], ra[0], rb[0], rb[0], rb[0], rc[0], rc[0], rc[0]);
        } else {
            int e = wpr - 1;
            ro[0] = life64(ra[e], ra[0], ra[1], rb[e], rb[0], rb[1], rc[e], rc[0], rc[1]);
            for (int j = 1; j < e; j++) /* interior: vectorisable */
                ro[j] = life64(ra[j - 1], ra[j], ra[j + 1], rb[j - 1], rb[j], rb[j + 1],
                               rc[j - 1], rc[j], rc[j + 1]);
            ro[e] = life64(ra[e - 1], ra[e], ra[0], rb[e - 1], rb[e], rb[0], rc[e - 1], rc[e],
                           rc[0]);
        }
        for (int j = 0; j < wpr; j++) c += __builtin_popcountll(ro[j]);
    }
    *count = c;
}

typedef struct {
    int wpr, h, y0, y1;
    const uint64_t *in;
    uint64_t *out;
    int64_t count;
} packed_task;

static void *packed_worker(void *arg) {
    packed_task *t = (packed_task *)arg;
    packed_rows(t->wpr, t->h, t->in, t->out, t->y0, t->y1, &t->count);
    return NULL;
}

/*
 * `turns` generations of a (64*wpr) x h torus held in `board` (updated in place).
 * counts (nullable, len turns): alive cells after each completed turn.
 */
int oracle_packed_run(int wpr, int h, uint64_t *board, long turns, int threads, int64_t *counts) {
    if (wpr <= 0 || h <= 0 || threads <= 0) return -1;
    size_t words = (size_t)wpr * h;
    uint64_t *tmp = (uint64_t *)malloc(words * sizeof(uint64_t));
    if (!tmp) return -2;
    if (threads > h) threads = h;
    packed_task *tasks = (packed_task *)calloc((size_t)threads, sizeof(packed_task));
    pthread_t *tids = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
    uint64_t *src = board, *dst = tmp;
    for (long t = 0; t < turns; t++) {
        for (int i = 0; i < threads; i++) {
            tasks[i].wpr = wpr; tasks[i].h = h;
            tasks[i].y0 = (int)((long)h * i / threads);
            tasks[i].y1 = (int)((long)h * (i + 1) / threads);
            tasks[i].in = src; tasks[i].out = dst;
            if (threads > 1) pthread_create(&tids[i], NULL, packed_worker, &tasks[i]);
            else packed_worker(&tasks[i]);
        }
        int64_t c = 0;
        for (int i = 0; i < threads; i++) {
            if (threads > 1) pthread_join(tids[i], NULL);
            c += tasks[i].count;
        }
        if (counts) counts[t] = c;
        uint64_t *x = src; src = dst; dst = x;
    }
    if (src != board) memcpy(board, src, words * sizeof(uint64_t));
    free(tmp); free(tasks); free(tids);
    return 0;
}

/* ------------------------------------------------------------------------------------ */
/* 3. Synthetic boards (the same definition libgolhip's on-device init implements)      */
/* ------------------------------------------------------------------------------------ */

static inline uint64_t splitmix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

/*
 * Random board, rows [y0, y1) of a width x height board, packed LSB-first into
 * wpr = width/64 words per row (width % 64 == 0).  Logical word i = y*wpr + j:
 *   density_q32 == 2^31 : word = splitmix64(seed + (i+1)*0x9E3779B97F4A7C15)
 *   otherwise           : cell (x,y) alive iff (uint32)splitmix64(seed + (c+1)*0x9E3779B97F4A7C15)
 *                         < density_q32, c = y*width + x.
 */
int oracle_init_random(int width, int y0, int y1, uint64_t seed, uint64_t density_q32,
                       uint64_t *out) {
    if (width % 64 != 0) return -1;
    int wpr = width / 64;
    const uint64_t g = 0x9E3779B97F4A7C15ULL;
    for (int y = y0; y < y1; y++) {
        for (int j = 0; j < wpr; j++) {
            uint64_t i = (uint64_t)y * wpr + j, w = 0;
            if (density_q32 == (1ULL << 31)) {
                w = splitmix64(seed + (i + 1) * g);
            } else {
                for (int b = 0; b < 64; b++) {
                    uint64_t c = (uint64_t)y * width + (uint64_t)j * 64 + b;
                    uint32_t d = (uint32_t)splitmix64(seed + (c + 1) * g);
                    if ((uint64_t)d < density_q32) w |= 1ULL << b;
                }
            }
            out[(size_t)(y - y0) * wpr + j] = w;
        }
    }
    return 0;
}
