// mgx_engine.hip -- MI355X (gfx950) kernels + C ABI (include/mgx.h) of the
// vectorised MiniGrid engine.
//
// HBM layout (engine-owned, struct-of-arrays, one row per env):
//   state   EnvState  [N]        16 B   agent/target/mission/episode scalars
//   grid    u8        [N][GS]    GS = roundup(S*S, 16), 1 B cell codes (mgx_device.h)
//   pcg     uint4     [N][2]     PCG64 state + increment (reset-only)
//   aux     uint4     [N]        {uinteger, has_uint32, mt_cursor lo, hi} (reset-only)
//   mt      u32       [L + pad]  shared MT19937(base_seed) output table
//   mtok    u8        [256][32]  TokenizeVocabWrapper tokens per mission id
// Caller-owned (torch tensors): the stacked observation, rewards, dones, ...
//
// Kernels (one env per lane, 64 envs per 256-thread workgroup):
//   mgx_step_kernel   step + render + frame-stack roll + fused auto-reset
//   mgx_reset_kernel  first seeded reset (SeedSequence -> PCG64 on device)
//   mgx_gae_kernel    GAE + advantage statistics
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/mgx.h"
#include "mgx_diag.h"
#include "mgx_device.h"

using namespace mgx;

namespace {

// Co-residency budget (per CU, while a refill epoch runs beside the steps): one refill wave per
// SIMD plus three step workgroups.  VGPRs per SIMD lane: 176 + 3 x 112 = 512 (granule 8), so
// the step kernel must stay at <= 112 VGPRs and the refill at <= 176.  LDS: 4 x refill
// (17.4 KB at the BASELINE configs) + 3 x step (25.8 KB) <= 160 KB.  Check with
// `make resource-usage` after any change to either kernel.
constexpr int BLOCK_ENVS = 64;
typedef uint16_t rpos_t;                    // episode ring positions (mod 2^16)
constexpr int MGX_MAX_RING = 4096;          // ring depth bound (a power of two, far below 2^16)
constexpr uint32_t NO_POP = 0xFFFFFFFFu;    // mgx_rollout_kernel: no pop this step
constexpr int MGX_NCOUNTERS = 32;          // [0..3] unused (per-workgroup slots), [4..7] step stamps, [8..] generator stamps
constexpr int BLOCK_THREADS = 256;
constexpr int FRAME = 147;                 // 3 x 7 x 7
constexpr int FRAME_DW4 = 147;             // dwords per env row at n_stack == 4 (588 B)
constexpr int FROW = 148;                  // LDS frame row (fast roll): byte 0 pad, bytes 1..147 frame
// MT19937 output ring (every env's CPython `random` is MT19937(seed) -- one shared
// stream read at per-env cursors, custom_env.py:82).  The ring holds groups [lo, hi) of the packed
// stream (mgx_device.h: ten 5-bit fields per group); hi * 10 words have been generated and `st` is
// the generator's state after them (a whole number of 624-word blocks).  No env ever reads below
// its oldest live cursor again -- the end of its current episode (cur_rng: a later VecEnv.reset()
// continues from there) or, in inline mode, that episode's start (start_rng: mgx_scene regenerates
// it) -- so mgx_mt_slide_kernel keeps the stream generated MT_AHEAD words past the furthest
// producer cursor, overwriting only dead groups (at most the ring's size above the oldest live
// cursor): the stream never runs out (round 2's host-built table of 2^24 words lasted ~1.1-1.5 M
// steps per env).  What the ring bounds is the SPREAD of the live cursors: every env reads the same
// stream at its own pace, and per-episode consumption is heavy-tailed (an abandoned live-locked
// attempt takes 4,096 words), so the spread grows like sqrt(steps) -- measured at GTG 8x8, 1,024
// envs: 74 k words after 4,900 steps.  The default ring (2^26 words) holds that spread for ~10^9
// steps per env at 65,536 envs; past it MGX_DEVERR_MT_TABLE is raised, never silent.
struct MtCtl {
    unsigned long long lo, hi;       // groups of the stream held by the ring
    unsigned long long span_min;     // min live cursor (words) of the running slide pass, ~0 between passes
    unsigned long long span_max;     // max producer cursor (words) of the running pass, 0 between passes
    unsigned int done;               // workgroups of the running pass that have reduced
    unsigned int pad;
    uint32_t st[624];                // MT19937 state at word hi * 10 (every output of it consumed)
    // refill production ceiling (mgx_refill_kernel): the episodes every env popped between the last two
    // refill launches, summed by the slide that follows the last one (running sum, result)
    unsigned long long cons_run, cons_last;
    // grid-wide ceiling of a refill wave's attempt rounds (round 4): round_cap episodes per env
    // for the next launch, from a fixed-point (1/1024) accumulator of the target production per epoch, so
    // that the ceiling alternates between floor and ceil of the target instead of always rounding up
    unsigned long long round_acc;
    int round_cap, round_pad;
    // prefix records (KParams.pfx): every stream position below rec_done has one (computed by the slide, a pass behind
    // the stream's generation: positions are read long after they are generated, MT_AHEAD)
    unsigned long long rec_done;
};
constexpr int MT_SB_WORDS = 3120;                         // lcm(624, 10): five MT blocks = 312 whole groups
constexpr int MT_SB_GROUPS = MT_SB_WORDS / MT_FIELDS;
constexpr int MT_SLIDE_MAX_SB = 64;                       // super-blocks one slide generates at most (200 k words)
constexpr unsigned long long MT_AHEAD = 1ull << 19;       // words kept generated past the furthest producer cursor
constexpr long long MT_HOST_FILL = 1ll << 20;             // words the host generates at create
// 256 threads: the slider must find room on a CU beside the step / rollout kernels (a 1,024-thread
// workgroup waited ~50 us for a whole CU behind the fused rollout, and the refill waited behind it)
constexpr int SLIDE_THREADS = 256, SLIDE_ENVS = 16 * SLIDE_THREADS;
// LDS bytes per resetting lane: MT window + objs list (obj_stride words, see mgx_create)
__host__ __device__ constexpr int scratch_per_env(int obj_stride, int nw) { return win_stride_of(nw) * 4 + obj_stride * 4; }

// ---- kernel clocks (mgx_set_clock; include/mgx.h).  Each launch of a clocked kernel records, per workgroup,
// its start and end in wall-clock ticks (s_memrealtime), so that a caller can time a kernel INSIDE a replayed
// hipGraph, beside whatever runs concurrently (bench.py's roofline: the timed region's own launches, not an eager
// probe); the launch's span is the min start to the max end over its workgroups.  No atomics: workgroup b of
// every launch of a class is the only writer of its own launch counter cnt[b] (every launch of a class has the
// same grid) and of its record of launch cnt[b] -- plain stores, one 16-B record per workgroup (a first version
// reduced with device-scope atomics on one address per launch and cost the 1,024-workgroup step kernel 48 us).
// Class block (u64): cnt[G], then [slots][G] records {start, end}; G = the class's grid (mgx_clock_groups).
// class 3 (round 6): the fused rollout's 32-env blocks (S = 16), whose grid is twice the step kernels' --
// every launch of a class must have the class's grid (workgroup b counts the launches it took part in)
enum { CLK_STEP = 0, CLK_REFILL = 1, CLK_SLIDE = 2, CLK_ROLL32 = 3, CLK_CLASSES = 4 };
struct KClock {
    unsigned long long *base[CLK_CLASSES];   // per class: cnt[G] then rec[slots][G][2]
    int groups[CLK_CLASSES];
    int slots;
};
struct KParams {
    EnvState *state;
    uint8_t *grid;
    uint4 *pcg;        // [N][2]
    uint4 *aux;        // [N]
    uint64_t *mt;                   // packed MT19937(seed) stream: ten 5-bit fields per group, a ring of
                                    // mt_mask+1 groups + MT_PAD mirror groups, extended by mgx_mt_slide_kernel
    const uint8_t *mtok;
    unsigned long long *counters;   // [0] steps [1] resets [2] livelocks [3] max cursor
    uint32_t *err;
    uint64_t mt_mask;               // ring slots - 1
    struct MtCtl *mtc;              // ring window + generator state (device)
    int64_t n;
    int64_t seed_base;              // base_seed + env_index_offset
    int S, GS, GSL, grid_lds, n_stack, img_bytes, stk_lds, stk_step, problem, cfg_mission, num_objects, all_doors_open;
    int obj_cap, obj_stride;        // generator objs list: capacity for this config, LDS words per lane (odd)
    uint32_t llw;
    int terminal_mode, mission64, fast_roll;
    int n_obstacles;        // floor((S-2)^2 * percent_obstacles) when cfg.obstacles (custom_env.py:156)
    int vis;                // see_through_walls == False: Grid.process_vis on every frame
    int has_move;           // the problem can draw 'move' missions: target_range words below are live
    int manual;             // PlaygroundEnv(manual=True): 'done' ends only a completed mission (custom_env.py:325)
    uint64_t *range_cur;    // [N]     target_range of the current episode (mgx_device.h: move_range)
    uint64_t *ring_range;   // [N][D]  ... of each queued episode
    // pre-generated episode ring (see mgx_refill_kernel): one REC-byte record per slot, slot = env * D + pos,
    //   [0, GS)        the grid
    //   [GS, GS+16)    header {ax|ay<<8|dir<<16|tx<<24, ty|ta<<8|mission<<16, livelocks, 0}
    //   [GS+16, GS+48) RNG snapshot after that episode's generation (PCG64 state; uinteger, has, MT cursor)
    //   then zeros to REC = roundup(GS + 48, 64): whole 64-B units, so the refill writes whole lines
    // (round 5: one array-of-records instead of grid / header+tokens / RNG arrays -- the refill's lanes wrote
    // their slots' 16-B pieces 16 KB apart, ~64 B of HBM write per 16-B store; the records are now written
    // by the whole wave, consecutive lanes on consecutive pieces.  The mission tokens are no longer copied
    // into the ring: the one reader, the SB3 layout's pop, looks them up in mtok.)
    uint8_t *ring_rec;      // [N][D][REC]
    int REC;
    uint4 *cur_rng;         // [N][2]   RNG snapshot after the current episode's generation
    // SPSC ring indices (rpos_t, mod 2^16; D is a power of two <= MGX_MAX_RING):
    rpos_t *ring_head;      // [N] consumer (step kernel) position
    rpos_t *ring_tail;      // [N] producer (refill kernel) position
    rpos_t *ring_pub;       // [N] ring_pubn as of the epoch's first per-step call: mgx_step_kernel pops below it
    rpos_t *ring_pubn;      // [N] ring_tail as the last COMPLETED refill left it, copied by the slide that follows
                            // it on the refill stream (a refill still running may have written ring_tail before
                            // its episodes reached another XCD's view; a completed one has released them):
                            // mgx_rollout_kernel pops below it, no copy on the steps' stream
    rpos_t *ring_seen;      // [N] ring_head as the last refill read it (its consumption estimate)
    uint32_t *fix_list;     // [N] envs whose ring was empty at their reset (mgx_fixup_kernel)
    uint32_t *fix_count;    // list length; fix_done: workgroups of the fixup kernel that finished
    uint32_t *fix_done;
    ulonglong4 *blk;        // [4 * nblk] per-workgroup stats: step/reset | fixup | refill waves (x2)
    int nblk;               // ceil(N / 64)
    int refill_epw;         // envs per refill wave at S = 8: 64, or 32 when 64-env waves leave SIMDs idle
    int D;
    int K;                  // refill epoch (steps)
    int cap;                // episodes an env produces per epoch beyond what the invariant needs (<0: fill to D)
    int initial_fill;       // this refill launch is mgx_reset's (fill every ring to D)
    int reset_mode;         // mgx_reset: 0 first (seeded, MT cursor 0), 1 seeded, 2 unseeded
    int refill_prio;        // s_setprio of the refill's waves (env MGX_REFILL_PRIO, 0..3)
    uint4 *start_rng;       // [N][2] inline mode only: RNG state at the start of the current episode's
                            //        generation (mgx_scene regenerates it), else null
    KClock clk;             // mgx_set_clock: kernel clocks (clk.slots == 0: off)
    // mgx_set_random_policy (ABI 7): the fused rollout draws its own actions when launched without any --
    // rnd_ctr[b] = random-policy launches rollout workgroup b has run (its sole writer); null: off
    unsigned long long *rnd_ctr;
    uint64_t rnd_seed;
    // multi-room problems with the ring (round 6): the MT-only generator prefix of every stream position, one u64
    // record per word -- [(group & mt_mask) * 10 + word], mgx_device.h pfx_pack -- or null
    uint64_t *pfx;
    int mt_shift;           // log2(ring groups): a position's wrap count is group >> mt_shift
};

// 16-B store, non-temporal (streaming: write-once data the kernel never reads back) when NT
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ void st16(uint4 *p, const uint4 v) {
    const u32x4_t w = {v.x, v.y, v.z, v.w};      // (one dwordx4 store either way: a HIP uint4 struct copied through a
    if (NT) __builtin_nontemporal_store(w, reinterpret_cast<u32x4_t *>(p));   // parameter compiled to four dword stores)
    else *reinterpret_cast<u32x4_t *>(p) = w;
}

__device__ __forceinline__ unsigned long long clk_now() { return (unsigned long long)wall_clock64(); }
__device__ __forceinline__ void clk_record(const KClock &k, int cls, unsigned long long t0) {   // one thread
    unsigned long long *c = k.base[cls];
    const int G = k.groups[cls], b = (int)blockIdx.x;
    const unsigned long long i = c[b];
    if (i < (unsigned long long)k.slots)
        reinterpret_cast<ulonglong2 *>(c + G)[i * (unsigned long long)G + b] = make_ulonglong2(t0, clk_now());
    c[b] = i + 1ull;
}

struct KOut {
    uint8_t *img, *dir;
    void *mis;
    uint8_t *t_img, *t_dir;
    void *t_mis;
    float *reward;
    double *reward64;
    uint8_t *term, *trunc, *done;
    float *ep_ret;
    int32_t *ep_len;
    int32_t *livelock;
};

// Grids: global rows are GS bytes (16-B multiple), LDS rows GSL = GS + 4 bytes
// (an odd number of dwords, so lane-private rows sit on distinct LDS banks).
__device__ __forceinline__ void grid_copy_in(uint8_t *lds, const uint8_t *g, int ne, int GS, int GSL) {
    const int q = GS >> 4;                              // 16-B chunks per row
    const uint4 *src = reinterpret_cast<const uint4 *>(g);
    for (int i = threadIdx.x; i < ne * q; i += BLOCK_THREADS) {
        const int e = i / q, c = i - e * q;
        const uint4 v = src[i];
        uint32_t *d = reinterpret_cast<uint32_t *>(lds + e * GSL + c * 16);
        d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
    }
}
__device__ __forceinline__ void grid_copy_out(uint8_t *g, const uint8_t *lds, int ne, int GS, int GSL,
                                              const uint8_t *dirty /* null = all */) {
    const int q = GS >> 4;
    uint4 *dst = reinterpret_cast<uint4 *>(g);
    for (int i = threadIdx.x; i < ne * q; i += BLOCK_THREADS) {
        const int e = i / q, c = i - e * q;
        if (dirty && !dirty[e]) continue;
        const uint32_t *s = reinterpret_cast<const uint32_t *>(lds + e * GSL + c * 16);
        dst[i] = make_uint4(s[0], s[1], s[2], s[3]);
    }
}

// A value every lane holds the same copy of (read from LDS) -> SGPRs
__device__ __forceinline__ unsigned long long wave_uniform64(unsigned long long v) {
    return ((unsigned long long)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
}

// Image-stack stores
__device__ __forceinline__ void stk_store(uint4 *p, uint4 v) { *p = v; }

// Mission-stack slot writer: slot `s` of env row gets mission tokens or zeros.
__device__ __forceinline__ void write_mission_slot(void *mis, int mission64, int64_t e, int n_stack, int s,
                                                   const uint8_t *tok /* null = zeros */) {
    uint4 t0 = make_uint4(0, 0, 0, 0), t1 = t0;
    if (tok) {
        t0 = reinterpret_cast<const uint4 *>(tok)[0];
        t1 = reinterpret_cast<const uint4 *>(tok)[1];
    }
    if (mission64) {
        longlong2 *r2 = reinterpret_cast<longlong2 *>(reinterpret_cast<int64_t *>(mis) + (e * n_stack + s) * 32);
        const uint32_t w[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const uint32_t word = w[k >> 1];
            const int sh = (k & 1) * 16;
            longlong2 v;
            v.x = (long long)((word >> sh) & 0xFF);
            v.y = (long long)((word >> (sh + 8)) & 0xFF);
            r2[k] = v;
        }
    } else {
        uint4 *row = reinterpret_cast<uint4 *>(reinterpret_cast<uint8_t *>(mis) + (e * n_stack + s) * 32);
        row[0] = t0;
        row[1] = t1;
    }
}

// One 16-B chunk of slot `s` of env e's mission stack: tokens (2 int64 or 16 u8 per
// chunk) or zeros.  Used by the step kernel's block-cooperative writer, so that one
// env's 1-KB (int64) stack row is written by consecutive threads, coalesced.
__device__ __forceinline__ void write_mission_chunk(void *mis, int mission64, int64_t e, int n_stack, int s, int c,
                                                    const uint8_t *tok /* null = zeros */) {
    if (mission64) {
        longlong2 v = make_longlong2(0, 0);
        if (tok) { v.x = tok[2 * c]; v.y = tok[2 * c + 1]; }
        reinterpret_cast<longlong2 *>(reinterpret_cast<int64_t *>(mis) + (e * n_stack + s) * 32)[c] = v;
    } else {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (tok) v = reinterpret_cast<const uint4 *>(tok)[c];
        reinterpret_cast<uint4 *>(reinterpret_cast<uint8_t *>(mis) + (e * n_stack + s) * 32)[c] = v;
    }
}

// Same, tokens given as two 16-byte halves (lane-linear LDS staging of the step kernel).
__device__ __forceinline__ void write_mission_chunk2(void *mis, int mission64, int64_t e, int n_stack, int s, int c,
                                                     const uint8_t *lo, const uint8_t *hi, bool zeros) {
    if (mission64) {
        longlong2 v = make_longlong2(0, 0);
        if (!zeros) {
            const uint8_t *h = c < 8 ? lo : hi;
            const int j = (2 * c) & 15;
            v.x = h[j]; v.y = h[j + 1];
        }
        reinterpret_cast<longlong2 *>(reinterpret_cast<int64_t *>(mis) + (e * n_stack + s) * 32)[c] = v;
    } else {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (!zeros) v = *reinterpret_cast<const uint4 *>(c == 0 ? lo : hi);
        reinterpret_cast<uint4 *>(reinterpret_cast<uint8_t *>(mis) + (e * n_stack + s) * 32)[c] = v;
    }
}

// Full mission stack for an episode holding `frames` frames (last `frames` slots set).
__device__ __forceinline__ void write_mission_stack(void *mis, int mission64, int64_t e, int n_stack, int frames,
                                                    const uint8_t *tok) {
    for (int s = 0; s < n_stack; s++) write_mission_slot(mis, mission64, e, n_stack, s, s >= n_stack - frames ? tok : nullptr);
}

// Direction stack roll: drop oldest one-hot, append newest (dir < 0: zeros).
__device__ __forceinline__ void dir_stack_roll(const uint8_t *src, uint8_t *dst, int64_t e, int n_stack, int newdir) {
    const int nb = 4 * n_stack;
    if (n_stack == 4) {
        uint4 v = reinterpret_cast<const uint4 *>(src)[e];
        uint32_t oh = newdir >= 0 ? (1u << (8 * newdir)) : 0u;
        uint4 o = make_uint4(v.y, v.z, v.w, oh);
        reinterpret_cast<uint4 *>(dst)[e] = o;
    } else {
        for (int k = 0; k < nb - 4; k++) dst[e * nb + k] = src[e * nb + 4 + k];   // forward: safe in place
        for (int k = 0; k < 4; k++) dst[e * nb + nb - 4 + k] = (uint8_t)(k == newdir);
    }
}
__device__ __forceinline__ void dir_stack_fresh(uint8_t *dst, int64_t e, int n_stack, int newdir) {
    const int nb = 4 * n_stack;
    if (n_stack == 4) {
        reinterpret_cast<uint4 *>(dst)[e] = make_uint4(0, 0, 0, 1u << (8 * newdir));
    } else {
        for (int k = 0; k < nb; k++) dst[e * nb + k] = (uint8_t)(k >= nb - 4 && (k - (nb - 4)) == newdir);
    }
}

template <int NW>
__device__ __forceinline__ void load_gen(Gen<NW> &G, const KParams &p, int64_t e, uint8_t *g, uint8_t *scratch, int lane) {
    G.g = g;
    G.S = p.S;
    G.table = p.mt;
    G.rmask = p.mt_mask;
    G.tlo = p.mtc->lo;              // uniform: scalar loads; the slider runs between kernels, never during
    G.thi = p.mtc->hi;
    // lane >= 0: workgroup LDS layout [64 windows][64 objs lists]; lane < 0: one env's private block
    constexpr int WS = win_stride<NW>();
    G.win = reinterpret_cast<uint64_t *>(scratch + (lane >= 0 ? lane * (WS * 4) : 0));
    G.objs = reinterpret_cast<uint32_t *>(scratch + (lane >= 0 ? BLOCK_ENVS * (WS * 4) + lane * (p.obj_stride * 4)
                                                               : WS * 4));
    G.llw = p.llw;
    G.err = 0;
    G.problem = p.problem;
    G.cfg_mission = p.cfg_mission;
    G.num_objects = p.num_objects;
    G.all_doors_open = p.all_doors_open;
    G.n_obstacles = p.n_obstacles;
    G.abort = false;
    G.phave = false;
    G.prec = 0;
    G.nobjs = 0;
    G.ax = G.ay = -1;
    G.adir = 0;
#if MGX_GEN_STAMPS
    G.stamps = p.counters;
    G.tlast = __builtin_amdgcn_s_memtime();
#endif
    gen_init(G);
}

template <int NW>
__device__ __forceinline__ void load_rng(Gen<NW> &G, const KParams &p, int64_t e) {
    uint4 s = p.pcg[2 * e], i = p.pcg[2 * e + 1], a = p.aux[e];
    G.pcg.sh = ((uint64_t)s.x << 32) | s.y;
    G.pcg.sl = ((uint64_t)s.z << 32) | s.w;
    G.pcg.ih = ((uint64_t)i.x << 32) | i.y;
    G.pcg.il = ((uint64_t)i.z << 32) | i.w;
    G.pcg.uinteger = a.x;
    G.pcg.has = a.y & 1u;           // bits 1..: abandoned attempts not yet reported (mgx_refill_kernel)
    G.cur = (uint64_t)a.z | ((uint64_t)a.w << 32);
    G.gbase = ~0ull >> 1;   // empty window
}
template <int NW>
__device__ __forceinline__ void store_rng(const Gen<NW> &G, const KParams &p, int64_t e, uint32_t pending_ll = 0) {
    p.pcg[2 * e] = make_uint4((uint32_t)(G.pcg.sh >> 32), (uint32_t)G.pcg.sh, (uint32_t)(G.pcg.sl >> 32), (uint32_t)G.pcg.sl);
    p.pcg[2 * e + 1] = make_uint4((uint32_t)(G.pcg.ih >> 32), (uint32_t)G.pcg.ih, (uint32_t)(G.pcg.il >> 32), (uint32_t)G.pcg.il);
    p.aux[e] = make_uint4(G.pcg.uinteger, G.pcg.has | (pending_ll << 1), (uint32_t)G.cur, (uint32_t)(G.cur >> 32));
}

template <int NW>
__device__ __forceinline__ void rng_snapshot(const Gen<NW> &G, uint4 *dst) {
    dst[0] = make_uint4((uint32_t)(G.pcg.sh >> 32), (uint32_t)G.pcg.sh, (uint32_t)(G.pcg.sl >> 32), (uint32_t)G.pcg.sl);
    dst[1] = make_uint4(G.pcg.uinteger, G.pcg.has, (uint32_t)G.cur, (uint32_t)(G.cur >> 32));
}
template <int NW>
__device__ __forceinline__ uint4 pack_hdr(const Gen<NW> &G, const ResetOut &R) {
    return make_uint4((uint32_t)G.ax | ((uint32_t)G.ay << 8) | ((uint32_t)G.adir << 16) | ((uint32_t)R.tx << 24),
                      (uint32_t)R.ty | ((uint32_t)R.ta << 8) | ((uint32_t)R.mission_id << 16),
                      (uint32_t)R.livelocks, 0u);
}

// Render the first frame of a fresh episode straight into the newest slot of the stack.
__device__ __forceinline__ void write_fresh_frame(const KParams &p, uint8_t *img, int64_t e, const uint8_t *g,
                                                  int ax, int ay, int dir) {
    uint8_t *dst = img + e * (int64_t)p.img_bytes + (p.img_bytes - FRAME);
    render_view(g, p.S, ax, ay, dir, 0, [&](int k, uint32_t v) {
        dst[k] = (uint8_t)v;
        dst[49 + k] = (uint8_t)(v >> 8);
        dst[98 + k] = (uint8_t)(v >> 16);
    });
    if (p.vis) apply_vis(dst);          // this thread's own global writes: read back coherently
}

// ============================================================== reset kernel
template <int NW, bool EXT>
__global__ __launch_bounds__(BLOCK_THREADS) void mgx_reset_kernel(KParams p, KOut o) {
    extern __shared__ __align__(16) uint8_t smem[];
    uint8_t *s_scr = smem;
    uint8_t *s_grid = smem + p.stk_lds;
    const int tid = threadIdx.x;
    const int64_t e0 = (int64_t)blockIdx.x * BLOCK_ENVS;
    const int ne = (int)min<int64_t>(BLOCK_ENVS, p.n - e0);
    __shared__ unsigned long long s_ll;
    __shared__ unsigned long long s_maxcur;
    __shared__ uint32_t s_err;
    if (tid == 0) { s_ll = 0; s_maxcur = 0; s_err = 0; }
    __syncthreads();
    if (tid < ne) {
        const int64_t e = e0 + tid;
        Gen<NW> G;
        load_gen(G, p, e, s_grid + tid * p.GSL, s_scr, tid);
        EnvState st;
        if (p.reset_mode == 0) {
            pcg_seed(G.pcg, (uint64_t)(p.seed_base + e));   // gymnasium Env.reset(seed=seed+i)
            G.cur = 0;                                       // random.seed(cfg.seed) in PlaygroundEnv.__init__
            st.reward_step = -1; st.mission_done = 0;
        } else {
            // Later VecEnv.reset(): both streams continue from the CURRENT episode (not from the
            // ring, which is discarded); mission_done / stored reward persist (Q2)
            const EnvState old = p.state[e];
            st.reward_step = old.reward_step; st.mission_done = old.mission_done;
            const uint4 c0 = p.cur_rng[2 * e], c1 = p.cur_rng[2 * e + 1], inc = p.pcg[2 * e + 1];
            if (p.reset_mode == 1) {
                pcg_seed(G.pcg, (uint64_t)(p.seed_base + e));
            } else {
                G.pcg.sh = ((uint64_t)c0.x << 32) | c0.y;
                G.pcg.sl = ((uint64_t)c0.z << 32) | c0.w;
                G.pcg.ih = ((uint64_t)inc.x << 32) | inc.y;
                G.pcg.il = ((uint64_t)inc.z << 32) | inc.w;
                G.pcg.uinteger = c1.x;
                G.pcg.has = c1.y;
            }
            G.cur = (uint64_t)c1.z | ((uint64_t)c1.w << 32);
        }
        G.gbase = ~0ull >> 1;
        if (p.start_rng) rng_snapshot(G, p.start_rng + 2 * e);
        ResetOut R;
        reset_env<NW, EXT>(G, R);
        if (G.nobjs > p.obj_cap) G.err |= 8u;   // objs list ran past its per-config capacity
        st.ax = (uint8_t)G.ax; st.ay = (uint8_t)G.ay; st.dir = (uint8_t)G.adir; st.carry = 0;
        st.step_count = 0;
        st.tx = R.tx; st.ty = R.ty; st.target_action = R.ta; st.mission_id = R.mission_id;
        st.frames = 1; st.flags = 0; st.pad = 0;
        p.state[e] = st;
        if (p.has_move) p.range_cur[e] = R.range;
        store_rng(G, p, e);
        rng_snapshot(G, p.cur_rng + 2 * e);
        p.ring_head[e] = 0; p.ring_tail[e] = 0; p.ring_pub[e] = 0; p.ring_pubn[e] = 0;   // empty ring
        p.ring_seen[e] = 0;
        // stacked obs: zeros + first frame
        uint8_t *row = o.img + e * (int64_t)p.img_bytes;
        for (int k = 0; k < p.img_bytes - FRAME; k++) row[k] = 0;
        write_fresh_frame(p, o.img, e, G.g, G.ax, G.ay, G.adir);
        dir_stack_fresh(o.dir, e, p.n_stack, G.adir);
        write_mission_stack(o.mis, p.mission64, e, p.n_stack, 1, p.mtok + R.mission_id * 32);
        if (o.livelock) o.livelock[e] = R.livelocks;
        atomicAdd(&s_ll, (unsigned long long)R.livelocks);
        atomicMax(&s_maxcur, (unsigned long long)G.cur);
        if (G.err) atomicOr(&s_err, G.err);
    }
    __syncthreads();
    grid_copy_out(p.grid + e0 * p.GS, s_grid, ne, p.GS, p.GSL, nullptr);
    if (tid == 0) {
        ulonglong4 b = p.blk[blockIdx.x];           // workgroup-private stats slot (no contention)
        b.y += (unsigned long long)ne; b.z += s_ll; b.w = b.w > s_maxcur ? b.w : s_maxcur;
        p.blk[blockIdx.x] = b;
        if (s_err) atomicOr(p.err, s_err);
    }
}

// Block barrier ordering LDS only.  __syncthreads() is a workgroup fence over every address space: each
// wave waits for ALL its vector-memory operations (vmcnt(0)) before the barrier -- the DMA wave for the
// episode prefetches it has just issued, the render waves for their row stores -- and the whole block
// waits with it.  In the rollout loop nothing crosses a barrier through global memory: the DMA wave's
// LDS-DMA fills are waited explicitly (s_waitcnt 0) before the end-of-step barrier, the stores are
// only read by later kernels.  (mgx_step_kernel likewise: its phase-1 loads are waited explicitly.)
// Used by mgx_step_kernel only: in mgx_rollout_kernel the full __syncthreads measured faster (same-box
// A/B, config 2: 6.8 vs 5.95 x 10^9 env-steps/s fused; per-step compact 5.08 vs 5.19 the other way round).
// An LDS-only fence does not do: LDS-DMA fills are LDS writes counted by vmcnt, so a release on LDS
// still waits for them.  Hence the barrier as inline asm -- lgkmcnt(0) (this wave's LDS reads and
// writes are done) and s_barrier -- with a memory clobber, so that the compiler moves no memory
// access across it.
__device__ __forceinline__ void sync_lds() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// The fused rollout's per-step barriers (MGX_ROLL_VMKEEP >= 0): LDS complete, at most N of this wave's vector
// memory operations still in flight (its row / output stores: nothing in the launch reads them back), then
// the barrier.  -1: __syncthreads(), a workgroup fence that waits for every store of the step.
template <int N>
__device__ __forceinline__ void sync_keep_vm() {
    if constexpr (N < 0) {
        __syncthreads();
    } else {
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
    }
}

// =============================================================== step kernel
// Grids in the step kernel's LDS are chunk-major, [GS/16][64 lanes][16 B] (the LDS-DMA
// layout: one 16-B chunk per lane per global_load_lds); byte b of lane le's grid:
template <int EPB = BLOCK_ENVS>   // envs per block (the chunk stride; the fused rollout also runs 32-env blocks)
__device__ __forceinline__ int cm_off(int le, int b) { return (b >> 4) * (EPB * 16) + le * 16 + (b & 15); }

// Render the view columns thread q (0..3) of env slot `le` owns -- vx = q and q + 4; thread 3
// only column 3, which holds the agent's own cell (3, 6) -- into a frame row fr ([type 49]
// [colour 49][state 49], cell c = vx*7 + vy).  The view is closed form: cell (vx, vy) = A +
// (6 - vy) * dir_vec + (vx - 3) * right_vec (minigrid's slice + (dir+1) rotate_left); (3, 6)
// -> carried object or None.  Out-of-grid cells are Wall, and so is every border cell of a
// grid (custom_env.py:132 wall_rect; no action can replace a wall), so a coordinate clamped
// as unsigned to S-1 (negative -> S-1, the far border) reads a Wall exactly when it is out of
// the grid: no bounds test, no select.
// Along a column the world cell moves by -dir_vec per vy (adds only, no multiplies).  `grids`
// is the block's current grids or its popped episodes' grids (both chunk-major).  Every grid
// byte is read before any frame byte is written: one LDS round trip.
template <int EPB = BLOCK_ENVS>
__device__ __forceinline__ void render_cols(const uint8_t *grids, int S, int le, int q, uint32_t rp, uint8_t *fr) {
    const int ax = rp & 0xFF, ay = (rp >> 8) & 0xFF, dir = (rp >> 16) & 3;
    const uint8_t carry = (uint8_t)(rp >> 24);
    const int dx = (dir == 0) - (dir == 2), dy = (dir == 1) - (dir == 3);
    const uint8_t *base = grids + le * 16;
    uint8_t code[2][7];
#pragma unroll
    for (int j = 0; j < 2; j++) {
        const int ox = q + 4 * j - 3;                                   // vx - 3 (column 7: unused)
        int wx = ax + 6 * dx - __mul24(ox, dy), wy = ay + 6 * dy + __mul24(ox, dx);
#pragma unroll
        for (int vy = 0; vy < 7; vy++) {
            const uint32_t cx = min((uint32_t)wx, (uint32_t)(S - 1)), cy = min((uint32_t)wy, (uint32_t)(S - 1));
            const int b = (int)__umul24(cy, (uint32_t)S) + (int)cx;
            code[j][vy] = base[b + __mul24(b >> 4, EPB * 16 - 16)];   // cm_off<EPB>(le, b)
            wx -= dx;
            wy -= dy;
        }
    }
    if (q == 3) code[0][6] = carry ? carry : CODE_EMPTY;
#pragma unroll
    for (int j = 0; j < 2; j++) {
        if (j == 1 && q == 3) break;
        const int c0 = 7 * (q + 4 * j);
#pragma unroll
        for (int vy = 0; vy < 7; vy++) {
            const uint32_t v = code[j][vy], t = v & 15u;
            fr[c0 + vy] = (uint8_t)(t == T_OPEN ? (uint32_t)T_DOOR : t);
            fr[49 + c0 + vy] = (uint8_t)__builtin_amdgcn_ubfe(v, 4, 3);
            fr[98 + c0 + vy] = (uint8_t)(t == T_DOOR ? 1u + (v >> 7) : 0u);
        }
    }
}

// A whole compact row (byte 0 direction, then the [type 49][colour 49][state 49] frame) of env slot `le`,
// written as dwords by its 4 threads (round 5; render_cols writes 43 single bytes per thread).  Two passes
// over the row's own LDS bytes, all four threads of an env being lanes of one wave (LDS operations of a wave
// complete in order):
//   1. each thread's columns as render_cols computes them, stored as cell CODES (1 byte per cell) at row
//      bytes 4 + c, c = vx * 7 + vy;
//   2. output dword k (row bytes 4k..4k+3) holds four consecutive cells of one plane whose codes are row
//      bytes 4k - B + 4 .. (B = 1, 50, 99: the plane's first byte), an unaligned window of two code dwords
//      with a per-plane constant shift (3, 2, 1): thread q's type dwords q + 4j, colour dwords 12 + q + 4j and
//      state dwords 24 + q + 4j (j < 3; and 36 for q = 0) all take their windows from code dwords q + 4j,
//      q + 4j + 1, read once.  The three dwords where planes meet (0: direction + types, 12: types + colours,
//      24: colours + state) are thread 0's.  Decoding is byte-parallel (SWAR) on the window:
//        t = code & 15; open door (11) -> door (4): t ^ 15 where (t & 0b1011) == 0b1011 (11 is the only such
//        type present); colour = (code >> 4) & 7; state = 1 + aux (bit 7) where t == 4 -- the one type with
//        (t & 0b1011) == 0 (no cell code is 0 here: 'unseen' exists only under see_through_walls=False, which
//        keeps render_cols + apply_vis) -- else 0.
//   All code reads of the wave are issued before its first output write (they share the row's bytes).
__device__ __forceinline__ uint32_t swar_type(uint32_t w) {
    const uint32_t t = w & 0x0F0F0F0Fu, m = ((w & 0x0B0B0B0Bu) + 0x05050505u) & 0x10101010u;
    return t ^ (m - (m >> 4));                       // 11 -> 11 ^ 15 = 4
}
__device__ __forceinline__ uint32_t swar_colour(uint32_t w) { return (w >> 4) & 0x07070707u; }
__device__ __forceinline__ uint32_t swar_state(uint32_t w) {
    const uint32_t door = ((((w & 0x0B0B0B0Bu) + 0x0F0F0F0Fu) & 0x10101010u) ^ 0x10101010u) >> 4;   // 0x01 per door byte
    return door + ((w >> 7) & door);                 // closed 1, locked 2
}
template <int EPB = BLOCK_ENVS>
__device__ __forceinline__ void render_row(const uint8_t *grids, int S, int le, int q, uint32_t rp, uint8_t *row) {
    const int ax = rp & 0xFF, ay = (rp >> 8) & 0xFF, dir = (rp >> 16) & 3;
    const uint8_t carry = (uint8_t)(rp >> 24);
    const int dx = (dir == 0) - (dir == 2), dy = (dir == 1) - (dir == 3);
    const uint8_t *base = grids + le * 16;
    uint8_t *cp = row + 4 + 7 * q;                                      // codes of column q (and q + 4)
#pragma unroll
    for (int j = 0; j < 2; j++) {
        if (j == 1 && q == 3) break;
        const int ox = q + 4 * j - 3;
        int wx = ax + 6 * dx - __mul24(ox, dy), wy = ay + 6 * dy + __mul24(ox, dx);
#pragma unroll
        for (int vy = 0; vy < 7; vy++) {
            const uint32_t cx = min((uint32_t)wx, (uint32_t)(S - 1)), cy = min((uint32_t)wy, (uint32_t)(S - 1));
            const int b = (int)__umul24(cy, (uint32_t)S) + (int)cx;
            uint8_t v = base[b + __mul24(b >> 4, EPB * 16 - 16)];      // cm_off<EPB>(le, b)
            if (j == 0 && vy == 6 && q == 3) v = carry ? carry : CODE_EMPTY;   // the agent's own cell
            cp[28 * j + vy] = v;
            wx -= dx;
            wy -= dy;
        }
    }
    asm volatile("" ::: "memory");                   // (compiler barriers: the hardware keeps a wave's LDS order)
    uint32_t *rw = reinterpret_cast<uint32_t *>(row);
    uint32_t c[8];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        c[2 * j] = rw[q + 4 * j];
        c[2 * j + 1] = rw[q + 4 * j + 1];
    }
    asm volatile("" ::: "memory");
    uint32_t ty[3], co[3], st[4];
#pragma unroll
    for (int j = 0; j < 3; j++) {
        ty[j] = swar_type(__builtin_amdgcn_alignbyte(c[2 * j + 1], c[2 * j], 3));
        co[j] = swar_colour(__builtin_amdgcn_alignbyte(c[2 * j + 1], c[2 * j], 2));
        st[j] = swar_state(__builtin_amdgcn_alignbyte(c[2 * j + 1], c[2 * j], 1));
    }
    st[3] = swar_state(__builtin_amdgcn_alignbyte(c[7], c[6], 1));
    if (q == 0) {
        // dword 0: direction, types of cells 0-2; 12: types 47, 48 (window of code dwords 12, 13), colours 0, 1;
        // 24: colours 46-48 (same window, shift 2), state 0
        ty[0] = (ty[0] & 0xFFFFFF00u) | (uint32_t)dir;
        co[0] = (co[0] & 0xFFFF0000u) | (swar_type(__builtin_amdgcn_alignbyte(c[7], c[6], 3)) & 0xFFFFu);
        st[0] = (st[0] & 0xFF000000u) | (swar_colour(__builtin_amdgcn_alignbyte(c[7], c[6], 2)) & 0x00FFFFFFu);
    }
#pragma unroll
    for (int j = 0; j < 3; j++) {
        rw[q + 4 * j] = ty[j];
        rw[12 + q + 4 * j] = co[j];
        rw[24 + q + 4 * j] = st[j];
    }
    if (q == 0) rw[36] = st[3];
}

// One env's MiniGridEnv.step + PlaygroundEnv.step (custom_env.py:269-330), as selects: every
// action's outcome is computed and the taken one kept (a branch per action made a divergent tree of
// exec-mask updates -- half of the phase's instructions were SALU mask bookkeeping).  The front
// cell is read from, and (pickup / drop / toggle) written to, env slot `le`'s chunk-major LDS grid.
struct StepRes {
    double rew;                       // the step's reward (Python float)
    uint32_t view;                    // ax | ay<<8 | dir<<16 | carry<<24: what gen_obs() saw -- before
                                      // PlaygroundEnv's key consumption (Q3)
    int sc, mdone, rs;                // step count, mission_done, stored-reward step (-1 = None)
    uint8_t carry;                    // carried object after the key consumption (Q4)
    bool term, trunc, done, dirty;    // dirty: the grid changed
};
template <int EPB = BLOCK_ENVS>
__device__ __forceinline__ StepRes env_step(const EnvState &st, int a, uint8_t *grids, int le, int S, int manual,
                                            uint64_t mrange) {
    StepRes R;
    const int ms = S * S;
    const int sc = st.step_count + 1;
    int ax = st.ax, ay = st.ay, dir = st.dir;
    uint8_t carry = st.carry;
    const int fx = ax + ((dir == 0) - (dir == 2)), fy = ay + ((dir == 1) - (dir == 3));
    uint8_t *fp = grids + cm_off<EPB>(le, fy * S + fx);
    const uint8_t fc = *fp;
    const int ft = fc & 15;
    // MiniGridEnv.step (3P)
    const bool isF = a == A_FORWARD, isT = a == A_TOGGLE;
    const int fcol = (fc >> 4) & 7;
    dir = (dir + (a == A_RIGHT) + 3 * (a == A_LEFT)) & 3;
    const bool mv = isF && can_overlap(fc);
    ax = mv ? fx : ax;
    ay = mv ? fy : ay;
    const bool goal = isF && ft == T_GOAL;
    const bool t0 = goal || (isF && ft == T_LAVA);
    const bool pick = a == A_PICKUP && can_pickup(fc) && carry == 0;
    const bool drop = a == A_DROP && ft == T_EMPTY && carry != 0;
    // toggle: a locked door opens only with a Key of its colour; an open door closes; a box turns
    // into its contents (the key it holds, or nothing)
    const bool t_door = isT && ft == T_DOOR && (!(fc >> 7) || ((carry & 15) == T_KEY && ((carry >> 4) & 7) == fcol));
    const bool t_open = isT && ft == T_OPEN, t_box = isT && ft == T_BOX;
    uint8_t nc = fc;
    nc = t_door ? mk_code(T_OPEN, fcol, 0) : nc;
    nc = t_open ? mk_code(T_DOOR, fcol, 0) : nc;
    nc = t_box ? ((fc >> 7) ? mk_code(T_KEY, fcol, 0) : CODE_EMPTY) : nc;
    nc = pick ? CODE_EMPTY : nc;
    nc = drop ? carry : nc;
    carry = pick ? fc : (drop ? (uint8_t)0 : carry);
    R.dirty = pick || drop || t_door || t_open || t_box;
    if (R.dirty) *fp = nc;
    R.trunc = sc >= ms;
    R.view = (uint32_t)ax | ((uint32_t)ay << 8) | ((uint32_t)dir << 16) | ((uint32_t)carry << 24);
    // ---- PlaygroundEnv.step (custom_env.py:269-330)
    const int md0 = st.mission_done, rs0 = st.reward_step;
    const bool is_gtg = st.mission_id == CMD_GOTOGOAL;
    // Q4: toggling a door while carrying anything of its colour consumes it (not on a terminating step)
    if (!t0 && isT && is_door(nc) && carry != 0 && ((nc >> 4) & 7) == ((carry >> 4) & 7)) carry = 0;
    // mission completed this step (each test only sets `reward_step` if unset, `done` flag)
    const int ta = st.target_action;
    const bool has_t = st.tx != NONE8, ta_fwd = ta != NONE8 && ta != 0;
    const int nfx = ax + ((dir == 0) - (dir == 2)), nfy = ay + ((dir == 1) - (dir == 3));
    // (bitwise & / |: short-circuit operators turned this into a nest of branches)
    const bool at_f = (nfx == st.tx) & (nfy == st.ty), at_a = (ax == st.tx) & (ay == st.ty);
    const bool hit = (!t0 & !md0) &
                     ((has_t & ta_fwd & at_f & (a == ta)) | (has_t & !ta_fwd & at_a) |
                      (!has_t & (ta != NONE8) & (a == ta)) |
                      ((st.mission_id >= MID_MOVE) & in_move_range(mrange, ax, ay)));
    const int md1 = hit ? 1 : md0, rs1 = (hit && rs0 < 0) ? sc : rs0;
    // 'done': the stored self.reward, or 0 -- in manual mode only a completed mission ends
    const bool dn = !t0 && a == A_DONE && (md1 || !manual);
    // reward: reaching the goal pays 1 - 0.9 sc/ms only on 'go to goal' missions; 'done' pays the
    // reward stored at mission completion
    double rew = 0.0;
    if ((goal && is_gtg) || (dn && md1)) rew = reward_at(t0 ? sc : rs1, ms);
    R.rew = rew;
    R.mdone = t0 ? (is_gtg ? md0 : 0) : (dn ? 0 : md1);
    R.rs = t0 ? (is_gtg ? rs0 : -1) : (dn ? -1 : rs1);
    R.term = t0 || dn;
    R.done = R.term || R.trunc;
    R.sc = sc;
    R.carry = carry;
    return R;
}

// One vectorised env step of 64 envs per 256-thread workgroup.  No RNG work
// happens here: auto-resets pop pre-generated episodes from the env's ring
// (mgx_refill_kernel); an empty ring defers the env to mgx_fixup_kernel, which
// runs right after on the same stream.  Keeping the generator out of this
// kernel keeps it register-light (high occupancy hides its memory latency).
// COMPACT: the compact rollout layout (mgx_step_compact) instead of the SB3 stacks -- each
// env's new observation is ONE 148-B row (byte 0 direction, bytes 1..147 the [c][vx][vy]
// frame: the fast path's LDS frame row, copied out verbatim) plus its mission id byte; no
// stack is read or rolled (mgx_gather rebuilds stacks from consecutive rows on demand).
template <typename ActT, bool COMPACT, int SC = 0>   // SC > 0: the grid size as a compile-time constant
__global__ __launch_bounds__(BLOCK_THREADS, 4) void mgx_step_kernel(KParams p, KOut o, const ActT *__restrict__ actions) {
    extern __shared__ __align__(16) uint8_t smem[];
    const int GS = SC > 0 ? ((SC * SC + 15) & ~15) : p.GS;
    // fast path (n_stack == 4) and COMPACT: smem = frame rows [64][148] (new frame at bytes
    // 1..147); staged path: smem = image stacks [64][IMG] (new frame in slot 0 of a row).
    const bool fast = !COMPACT && p.fast_roll;
    uint8_t *s_stk = smem;
    // COMPACT keeps no token staging and only [64][148] frame rows: 20.3 KB at S=8, so four step
    // workgroups fit beside the refill's four waves in a CU's 160 KB (4 x 20.3 + 4 x 17.4); with
    // the SB3 layout's 25.8 KB only three did, and the fourth waited for a second round
    constexpr int CSTK = (BLOCK_ENVS * FROW + 15) & ~15;
    uint8_t *s_grid = smem + (COMPACT ? CSTK : p.stk_step);   // grids, chunk-major [GS/16][64 lanes][16 B] (cm_off)
    uint8_t *s_pgrid = s_grid + BLOCK_ENVS * GS;   // popped episodes' grids, same layout
    // LDS-DMA destinations are lane-linear (kept in the dynamic segment: hipcc 7.2 emitted no
    // M0 setup for a static __shared__ destination)
    uint4 *s_phdr = reinterpret_cast<uint4 *>(s_pgrid + BLOCK_ENVS * GS);   // popped ring slot header
    uint4 *s_tokA = s_phdr + BLOCK_ENVS;         // per lane: the current mission's tokens 0..15,
    uint4 *s_tokB = s_tokA + BLOCK_ENVS;         // 16..31 (envs whose stack is still filling)
    uint4 *s_prng = COMPACT ? s_phdr + BLOCK_ENVS : s_tokB + BLOCK_ENVS;    // [2][64] popped RNG snapshot
                                                 // (s_tokA / s_tokB: none in COMPACT)
    const int IMG = p.img_bytes;
    const int FSTRIDE = (fast || COMPACT) ? FROW : IMG, FOFF = (fast || COMPACT) ? 1 : 0;
    __shared__ uint32_t s_rp[BLOCK_ENVS];        // render params ax | ay<<8 | dir<<16 | carry<<24
    __shared__ uint8_t s_done[BLOCK_ENVS];
    __shared__ uint8_t s_term[BLOCK_ENVS];       // done env whose stacked terminal_observation is written
    __shared__ uint8_t s_dlist[BLOCK_ENVS];      // envs that popped a new episode (render + mission lists)
    __shared__ uint8_t s_flist[BLOCK_ENVS];      // envs whose mission stack is still filling
    __shared__ uint8_t s_fslot[BLOCK_ENVS];      // ... and the slot that flips 0 -> tokens
    __shared__ uint8_t s_popf[BLOCK_ENVS];       // env popped a new episode (its grid is in s_pgrid)
    __shared__ int s_nd, s_npop, s_nf;
    __shared__ unsigned long long s_dmask, s_tmask;   // done / terminal-written envs as bit masks
    __shared__ unsigned long long s_dirtym;           // envs whose grid changed
    __shared__ unsigned long long s_ll;

    const int tid = threadIdx.x;
    const int64_t e0 = (int64_t)blockIdx.x * BLOCK_ENVS;
    const int ne = (int)min<int64_t>(BLOCK_ENVS, p.n - e0);
    const int S = SC > 0 ? SC : p.S;
    if (tid == 0) s_ll = 0;
    __shared__ unsigned long long s_t0;           // kernel clock: this workgroup's start
    if (p.clk.slots && tid == 0) s_t0 = clk_now();
#if MGX_STAMPS
    const unsigned long long ts0 = __builtin_amdgcn_s_memtime();
    unsigned long long ts1 = 0, ts2 = 0, tsA = 0, tsB = 0, tsC = 0;
#endif

    // ---- phase 1: issue every load up front (one round trip; wave 0's pop: a second) ----
    EnvState st;
    int a = 0;
    uint4 odir = make_uint4(0, 0, 0, 0);          // old direction stack (n_stack == 4: one uint4)
    rpos_t rhead = 0, rpub = 0;                   // this env's ring position and published end
    uint64_t mrange = 0;                          // 'move' target_range (problems mov / full only)
    // (a) fast roll: the old image-stack dwords this lane's output quads need, into registers
    constexpr int DW = FRAME_DW4;                                                     // 147
    constexpr int MAXQ = (BLOCK_ENVS * DW / 4 + BLOCK_THREADS - 1) / BLOCK_THREADS;  // 10
    const uint32_t *g32in = reinterpret_cast<const uint32_t *>(o.img + e0 * (int64_t)IMG);
    const int limit = ne * DW;
    const int nq = fast ? (limit >> 2) : 0;
    uint4 qa[MAXQ];
    uint32_t qb[MAXQ];
    if (fast) {
#pragma unroll
        for (int r = 0; r < MAXQ; r++) {
            const int q = r * BLOCK_THREADS + tid, k = 4 * q;
            qa[r] = make_uint4(0, 0, 0, 0);
            qb[r] = 0;
            // quads wholly inside a row's new-frame columns (111..146) need no old data:
            // skipping them saves the dropped oldest frame's 147 B per env of reads
            const int j0 = k - (k / DW) * DW;
            if (q < nq && !(j0 >= 111 && j0 <= DW - 4)) {
                if (k + 39 < limit) {
                    qa[r] = *reinterpret_cast<const uint4 *>(g32in + k + 36);          // 16-B aligned
                } else {                                                               // last row: stay inside
                    if (k + 36 < limit) qa[r].x = g32in[k + 36];
                    if (k + 37 < limit) qa[r].y = g32in[k + 37];
                    if (k + 38 < limit) qa[r].z = g32in[k + 38];
                }
                if (k + 40 < limit) qb[r] = g32in[k + 40];
            }
        }
    }
    // ... and for the tail dword of a partial block (not a multiple of 4 dwords)
    const int kt = nq * 4 + tid;
    uint32_t tq36 = 0, tq37 = 0;
    if (fast && kt < limit) {
        tq36 = g32in[kt + 36];
        if (kt + 37 < limit) tq37 = g32in[kt + 37];
    }
    // (b) staged path: the whole old stacks -> LDS
    if (!fast && !COMPACT) {
        const uint8_t *gimg = o.img + e0 * (int64_t)IMG;
        const int nbytes = ne * IMG;
        const int n16 = nbytes >> 4;
        const uint4 *src = reinterpret_cast<const uint4 *>(gimg);
        uint4 *dst = reinterpret_cast<uint4 *>(s_stk);
        for (int i = tid; i < n16; i += BLOCK_THREADS) dst[i] = src[i];
        for (int i = (n16 << 4) + tid; i < nbytes; i += BLOCK_THREADS) s_stk[i] = gimg[i];
    }

    // (c) env state, action, direction row and ring indices of env (tid mod 64).  Every wave
    // loads them (three of the four copies are L2 hits) so that the loads are branch-free: a
    // phi copy at the end of a `tid < ne` branch would force a wait before the grid DMA.
    {
        const int le0 = min(tid & (BLOCK_ENVS - 1), ne - 1);
        const uint4 sv = reinterpret_cast<const uint4 *>(p.state)[e0 + le0];
        __builtin_memcpy(&st, &sv, sizeof st);
        a = (int)actions[e0 + le0];
        odir = (!COMPACT && p.n_stack == 4) ? reinterpret_cast<const uint4 *>(o.dir)[e0 + le0]
                                            : reinterpret_cast<const uint4 *>(p.state)[0];      // unused
        rhead = p.ring_head[e0 + le0];           // allocated (zeros) even without a ring
        rpub = p.ring_pub[e0 + le0];
        mrange = p.range_cur[p.has_move ? e0 + le0 : 0];
    }
    // (d) grids -> LDS by LDS-DMA (no registers, nothing to wait on before the barrier):
    // wave w moves chunks w, w+4, ... of all 64 envs, one env per lane.  After the register
    // loads: hipcc waits vmcnt(0) at the next use of a register load while an LDS-DMA is in
    // flight, which would serialise them.
    {
        const int lane = tid & (BLOCK_ENVS - 1);
        const uint4 *src = reinterpret_cast<const uint4 *>(p.grid + (e0 + min(lane, ne - 1)) * GS);
        for (int c = tid >> 6; c < (GS >> 4); c += BLOCK_THREADS / 64)
            __builtin_amdgcn_global_load_lds(src + c, s_grid + c * (BLOCK_ENVS * 16), 16, 0, 0);
    }
    // (e) SubprocVecEnv auto-reset, speculatively.  A step can end the episode only on
    // 'forward' (goal / lava ahead), on 'done' or at the time limit, which the state and the
    // action alone tell (every wave holds them for env tid mod 64); for those envs the next
    // pre-generated episode (header, tokens, grid, RNG snapshot) is fetched, and used only if
    // the step does end it.  Envs whose stack is still filling fetch their mission's tokens.
    // This second round trip depends on the first, so WAVE 1 issues it and goes on to the
    // barrier without waiting: its latency runs under wave 0's step logic, and only the pop
    // (after the post-logic barrier, which wave 1 reaches once the DMA has landed) reads it.
    const bool spec = p.D > 0 && (a == A_FORWARD || a == A_DONE || st.step_count + 1 >= S * S) &&
                      (rpos_t)(rpub - rhead) != 0;
    const bool wave1 = (tid >> 6) == 1;
    // Every phase-1 load of this wave has landed (register loads and LDS-DMA alike).  Saying
    // so explicitly matters: otherwise the waitcnt pass assumes a qa/qb load may be pending
    // on some path and puts a vmcnt(0) before every roll quad of phase 3, which then waits
    // on the previous quad's STORES (vmcnt counts both) and serialises the whole roll.
    __builtin_amdgcn_s_waitcnt(0);
    if (wave1) {
        const int lw = tid - BLOCK_ENVS;
        if (lw < ne) {
            if (!COMPACT && st.frames < p.n_stack) {
                const uint4 *t = reinterpret_cast<const uint4 *>(p.mtok + st.mission_id * 32);
                __builtin_amdgcn_global_load_lds(t, s_tokA, 16, 0, 0);
                __builtin_amdgcn_global_load_lds(t + 1, s_tokB, 16, 0, 0);
            }
            if (spec) {
                const int64_t slot = (e0 + lw) * p.D + (rhead & (p.D - 1));
                const uint4 *rec = reinterpret_cast<const uint4 *>(p.ring_rec + slot * (SC > 0 ? ((GS + 48 + 63) & ~63) : p.REC));
                __builtin_amdgcn_global_load_lds(rec + (GS >> 4), s_phdr, 16, 0, 0);
                __builtin_amdgcn_global_load_lds(rec + (GS >> 4) + 1, s_prng, 16, 0, 0);
                __builtin_amdgcn_global_load_lds(rec + (GS >> 4) + 2, s_prng + BLOCK_ENVS, 16, 0, 0);
                for (int c = 0; c < (GS >> 4); c++)
                    __builtin_amdgcn_global_load_lds(rec + c, s_pgrid + c * (BLOCK_ENVS * 16), 16, 0, 0);
            }
            // (no register load here: its phi copy after the branch would wait on the DMA above)
        }
    }
    sync_lds();
#if MGX_STAMPS
    ts1 = __builtin_amdgcn_s_memtime();
#endif

    // ---- phase 2a: one lane per env: MiniGridEnv.step + PlaygroundEnv.step
    uint32_t my_err = 0;
    int new_head = -1;
    bool done = false, term = false, trunc = false, dirty = false, fill = false, popped = false;
    int mdone = 0, rs = -1, dir = 0;
    // the block waits for wave 0's logic at the next barrier: MGX_STEP_LOGIC_PRIO raises its issue priority for
    // the phase (over the co-resident refill waves' 2), back to 0 after the ballot compaction below
    if (MGX_STEP_LOGIC_PRIO && tid < BLOCK_ENVS) {
        if (MGX_STEP_LOGIC_PRIO == 3) __builtin_amdgcn_s_setprio(3);
        else if (MGX_STEP_LOGIC_PRIO == 2) __builtin_amdgcn_s_setprio(2);
        else __builtin_amdgcn_s_setprio(1);
    }
    if (tid < ne) {
        const int64_t e = e0 + tid;
        if ((unsigned)a > 6u) { my_err |= MGX_DEVERR_BAD_ACTION; a = -1; }
        const StepRes r = env_step(st, a, s_grid, tid, S, p.manual, mrange);
        const int ax = r.view & 0xFF, ay = (r.view >> 8) & 0xFF;
        const uint8_t carry = r.carry;
        dir = (r.view >> 16) & 3;
        s_rp[tid] = r.view;
        const double rew = r.rew;
        const int sc = r.sc;
        term = r.term; trunc = r.trunc; done = r.done; dirty = r.dirty; mdone = r.mdone; rs = r.rs;
        // the episode ends (auto-reset) only on 'forward' into goal / lava, on 'done' or at the time
        // limit, each of which implies `spec`: the next episode is already in LDS (phase 1e)
        const bool avail = done && spec;
        const bool filling = !COMPACT && !done && st.frames < p.n_stack;
        const bool tw = done && (p.terminal_mode == MGX_TERMINAL_ALL ||
                                 (p.terminal_mode == MGX_TERMINAL_TRUNCATED && trunc && !term));
        if (tw && !COMPACT) {                          // stacked terminal_observation: dir + mission
            // (rare; before the pop rewrites this env's direction row)
            const int frames = min((int)st.frames + 1, p.n_stack);
            if (p.n_stack == 4)
                reinterpret_cast<uint4 *>(o.t_dir)[e] = make_uint4(odir.y, odir.z, odir.w, 1u << (8 * dir));
            else
                dir_stack_roll(o.dir, o.t_dir, e, p.n_stack, dir);
            write_mission_stack(o.t_mis, p.mission64, e, p.n_stack, frames, p.mtok + st.mission_id * 32);
            // leave no load of this rare path pending in the waitcnt pass's view: otherwise it
            // puts a vmcnt(0) (which waits on every STORE in flight) before the mission writer
            __builtin_amdgcn_s_waitcnt(0);
        }
        if (avail) {                                 // the pop itself follows the next barrier
            new_head = (int)(rpos_t)(rhead + 1);    // published after a barrier, loads consumed
            dirty = true;
            popped = true;
        } else if (done && p.D > 0) {
            my_err |= MGX_DEVERR_RING_EMPTY;   // cannot happen (refill production rule)
        } else if (done) {
            // no ring: mgx_fixup_kernel generates this env's episode inline.  Keep the
            // episode-spanning flags (Q2) in the state it will complete.
            st.reward_step = (int16_t)rs; st.mission_done = (uint8_t)mdone;
            p.state[e] = st;
            p.fix_list[atomicAdd(p.fix_count, 1u)] = (uint32_t)e;
        }
        o.reward[e] = (float)rew;
        if (o.reward64) o.reward64[e] = rew;
        o.term[e] = term;
        o.trunc[e] = trunc;
        if (o.done) o.done[e] = done;
        if (o.ep_ret) o.ep_ret[e] = (float)rew;       // only the final step can pay a reward
        if (o.ep_len) o.ep_len[e] = sc;
        if (!done) {
            const int frames = min((int)st.frames + 1, p.n_stack);
            if (COMPACT)
                static_cast<uint8_t *>(o.mis)[e] = st.mission_id;
            else if (p.n_stack == 4)
                reinterpret_cast<uint4 *>(o.dir)[e] = make_uint4(odir.y, odir.z, odir.w, 1u << (8 * dir));
            else
                dir_stack_roll(o.dir, o.dir, e, p.n_stack, dir);
            if (filling) {                             // stack still filling: one slot flips 0 -> mission
                fill = true;
                s_fslot[tid] = (uint8_t)(p.n_stack - frames);
            }
            st.ax = (uint8_t)ax; st.ay = (uint8_t)ay; st.dir = (uint8_t)dir; st.carry = carry;
            st.step_count = (uint16_t)sc; st.reward_step = (int16_t)rs; st.mission_done = (uint8_t)mdone;
            st.frames = (uint8_t)frames;
            p.state[e] = st;
            if (o.livelock) o.livelock[e] = 0;
        }
        s_done[tid] = done;
        s_term[tid] = tw;
        s_popf[tid] = popped;
    } else if (tid < BLOCK_ENVS) {
        s_done[tid] = 0;
        s_term[tid] = 0;
        s_popf[tid] = 0;
    }
    if (tid < BLOCK_ENVS) {                            // wave 0: ballot compaction of the lists
        const unsigned long long fm = __ballot(fill), dm = __ballot(done), pm = __ballot(popped);
        const unsigned long long tm = __ballot(tid < ne && s_term[tid]), gm = __ballot(dirty);
        if (fill) s_flist[__popcll(fm & __lanemask_lt())] = (uint8_t)tid;
        if (popped) s_dlist[__popcll(pm & __lanemask_lt())] = (uint8_t)tid;
        if (tid == 0) {
            s_nf = __popcll(fm); s_nd = __popcll(dm); s_npop = __popcll(pm); s_dmask = dm; s_tmask = tm;
            s_dirtym = gm;
        }
        if (MGX_STEP_LOGIC_PRIO) __builtin_amdgcn_s_setprio(0);
    }
    if (my_err) atomicOr(p.err, my_err);
    if (wave1) __builtin_amdgcn_s_waitcnt(0);          // the auto-reset prefetch has landed in LDS
    sync_lds();
    // SubprocVecEnv auto-reset: the env takes the popped episode (its header and RNG snapshot
    // were prefetched by wave 1 under the step logic).
    if (popped) {
        const int64_t e = e0 + tid;
        const uint4 h = s_phdr[tid];
        p.cur_rng[2 * e] = s_prng[tid];
        p.cur_rng[2 * e + 1] = s_prng[BLOCK_ENVS + tid];
        if (p.has_move) p.range_cur[e] = p.ring_range[e * p.D + (rhead & (p.D - 1))];
        const int ndir = (h.x >> 16) & 0xFF;
        const uint8_t mid = (uint8_t)(h.y >> 16);
        EnvState ns;
        ns.ax = (uint8_t)(h.x & 0xFF); ns.ay = (uint8_t)((h.x >> 8) & 0xFF); ns.dir = (uint8_t)ndir; ns.carry = 0;
        ns.step_count = 0; ns.reward_step = (int16_t)rs;          // survives the reset (Q2)
        ns.tx = (uint8_t)(h.x >> 24); ns.ty = (uint8_t)h.y; ns.target_action = (uint8_t)(h.y >> 8);
        ns.mission_id = mid;
        ns.mission_done = (uint8_t)mdone; ns.frames = 1; ns.flags = 0; ns.pad = 0;
        p.state[e] = ns;
        if (COMPACT) static_cast<uint8_t *>(o.mis)[e] = mid;
        else dir_stack_fresh(o.dir, e, p.n_stack, ndir);
        if (o.livelock) o.livelock[e] = (int)h.z;
        if (h.z) atomicAdd(&s_ll, (unsigned long long)h.z);
    }
    // ring heads: the popped slot is consumed (its DMA landed in phase 1), so the refill may
    // reuse it.  Every lane writes its head, changed or not: one 64-B store per block instead
    // of a byte store per popped env.
    if (tid < ne && p.D > 0) p.ring_head[e0 + tid] = (rpos_t)(new_head >= 0 ? new_head : rhead);
    // ---- phase 5 (issued here, before the render, so the stores drain under it): write back
    // the grids that changed (moves, pickups, resets; a popped env's new grid is in the staging
    // area, both chunk-major), at line granularity: grids smaller than a 128-B line are written
    // for every env of a line with a dirty grid, so that no line is written in part.
    if (!(MGX_DIAG_SKIP & 16)) {
        const int q16 = GS >> 4;
        const int epl = GS < 128 ? 128 / GS : 1;          // envs per line (GS is a multiple of 16)
        const unsigned long long dirtym = s_dirtym;
        uint4 *dst = reinterpret_cast<uint4 *>(p.grid + e0 * GS);
        for (int i = tid; i < ne * q16; i += BLOCK_THREADS) {
            const int e = i / q16, c = i - e * q16;
            if (!((dirtym >> (e & ~(epl - 1))) & ((1ull << epl) - 1))) continue;
            dst[i] = *reinterpret_cast<const uint4 *>((s_popf[e] ? s_pgrid : s_grid) + c * (BLOCK_ENVS * 16) + e * 16);
        }
    }

#if MGX_STAMPS
    tsA = __builtin_amdgcn_s_memtime();
#endif
    // ---- phase 2b: mission stacks first (their stores drain during the render), block-
    // cooperative and coalesced: fresh stacks of popped envs (zeros + tokens in the newest
    // slot), then the one flipping slot of filling envs
    if (!COMPACT) {
        const int K = p.n_stack, CPS = p.mission64 ? 16 : 2, per = K * CPS;
        const int tot_d = s_npop * per;
        for (int w = tid; w < tot_d; w += BLOCK_THREADS) {
            const int i = w / per, j = w - i * per;
            const int le = s_dlist[i], sl = j / CPS, c = j - sl * CPS;
            // the popped episode's tokens: its mission id (header) -> the token table (L2-resident; round 5: the
            // ring no longer carries a copy of them)
            const uint8_t *tk = p.mtok + ((s_phdr[le].y >> 16) & 0xFFu) * 32;
            if (!(MGX_DIAG_SKIP & 4)) write_mission_chunk2(o.mis, p.mission64, e0 + le, K, sl, c, tk, tk + 16, sl != K - 1);
        }
        const uint8_t *tA = reinterpret_cast<const uint8_t *>(s_tokA), *tB = reinterpret_cast<const uint8_t *>(s_tokB);
        // int64: the flipping slot (256 B, whole lines); u8: the whole row (one line at n_stack
        // 4; a 32-B slot alone would be a partial-line write)
        const int perf = p.mission64 ? CPS : per, tot_f = s_nf * perf;
        for (int w = tid; w < tot_f; w += BLOCK_THREADS) {
            const int i = w / perf, j = w - i * perf;
            const int le = s_flist[i], fs = s_fslot[le];
            const int sl = p.mission64 ? fs : j / CPS, c = p.mission64 ? j : j - (j / CPS) * CPS;
            if (!(MGX_DIAG_SKIP & 4)) write_mission_chunk2(o.mis, p.mission64, e0 + le, K, sl, c, tA + le * 16, tB + le * 16, sl < fs);
        }
    }
    // ---- phase 2c (rare, block-uniform): the terminal frame of every env whose stacked
    // terminal_observation is written (the finished episode's post-step view) is rendered
    // into the env's newest-frame LDS slot -- free until the render below -- and copied out
    // as the terminal stack's newest slot.  No LDS of its own: the step kernel's LDS is what
    // keeps three of its workgroups co-resident with the refill's waves on a CU.
    if (s_tmask) {
        {
            const int le = tid >> 2, q = tid & 3;
            if (le < ne && s_term[le]) {
                if (COMPACT && !p.vis) render_row(s_grid, S, le, q, s_rp[le], s_stk + le * FROW);   // (whole row)
                else render_cols(s_grid, S, le, q, s_rp[le], s_stk + le * FSTRIDE + FOFF);
            }
        }
        sync_lds();
        if (p.vis) {
            if (tid < ne && s_term[tid]) apply_vis(s_stk + tid * FSTRIDE + FOFF);
            sync_lds();
        }
        if (COMPACT) {                                // terminal row: byte 0 direction, then the frame
            if (tid < ne && s_term[tid]) s_stk[tid * FROW] = (uint8_t)((s_rp[tid] >> 16) & 3);
            sync_lds();
            const int le = tid >> 2, q = tid & 3;
            if (le < ne && s_term[le]) {
                const uint32_t *fr = reinterpret_cast<const uint32_t *>(s_stk + le * FROW);
                uint32_t *t = reinterpret_cast<uint32_t *>(o.t_img + (e0 + le) * (int64_t)FROW);
#pragma unroll 1
                for (int k = 10 * q; k < min(10 * q + 10, FROW / 4); k++) t[k] = fr[k];
            }
        } else {
            const int le = tid >> 2, q = tid & 3;
            if (le < ne && s_term[le]) {
                const uint8_t *fr = s_stk + le * FSTRIDE + FOFF;
                uint8_t *t = o.t_img + (e0 + le) * (int64_t)IMG + (IMG - FRAME);
#pragma unroll 1
                for (int k = 37 * q; k < min(37 * q + 37, FRAME); k++) t[k] = fr[k];
            }
        }
        sync_lds();
    }
    // ---- phase 2c: one render pass for the whole block (all 256 threads, 4 per env): the
    // newest frame of every env -- the first frame of the new episode where one was popped
    // (rendered straight from its staged grid).
    {
        const int le = tid >> 2, q = tid & 3;
        if (le < ne) {
            const bool pop = s_popf[le];
            const uint32_t rp = pop ? (s_phdr[le].x & 0xFFFFFFu) : s_rp[le];   // popped: ax | ay<<8 | dir<<16
            if (COMPACT && !p.vis) {                  // the whole row as dwords, direction included (render_row)
                render_row(pop ? s_pgrid : s_grid, S, le, q, rp, s_stk + le * FROW);
            } else {
                render_cols(pop ? s_pgrid : s_grid, S, le, q, rp, s_stk + le * FSTRIDE + FOFF);
                if (COMPACT && q == 0) s_stk[le * FROW] = (uint8_t)((rp >> 16) & 3);   // row byte 0: direction
            }
        }
    }
    // COMPACT without process_vis: each wave copies out the 16 rows it rendered itself (below),
    // no block barrier -- the waves leave the lock-step here
    const bool wave_rows = COMPACT && !p.vis;
    if (!wave_rows) sync_lds();
    if (p.vis) {                                       // see_through_walls=False: process_vis
        if (tid < ne) apply_vis(s_stk + tid * FSTRIDE + FOFF);
        sync_lds();
    }
#if MGX_STAMPS
    tsB = __builtin_amdgcn_s_memtime();
#endif
    const int nd = s_nd;
    // ---- phase 2d (staged path): the older slots of each written terminal_observation
    // (the fast path writes them in phase 3 from registers)
    if (s_tmask && !fast && !COMPACT) {
        const int le = tid >> 2, q = tid & 3;
        if (le < ne && s_term[le]) {
            uint8_t *t = o.t_img + (e0 + le) * (int64_t)IMG;
            const uint8_t *old = s_stk + le * IMG;
            for (int off = q; off < IMG - FRAME; off += 4) t[off] = old[off + FRAME];
        }
    }
#if MGX_STAMPS
    ts2 = __builtin_amdgcn_s_memtime();
#endif

    // ---- phase 3: roll the image stacks.  out byte o of an env row = its old byte o+147
    // (o < IMG-147) or the newest frame (o >= IMG-147); done envs: zeros + newest frame.
    // Every quad is stored once, here: an earlier version stored the rows' old part right
    // after phase 1 and the rest here, so the 128-B lines across each row's seam were written
    // in two halves far apart in time; on MI355X that took 36 us per step instead of 27.
    if (COMPACT) {
        // rows are contiguous in LDS and in the output: coalesced copies, per wave (its 16 rows,
        // 2,368 B, 16-B aligned) or, after a block barrier, per block
        const int r0 = wave_rows ? (tid >> 6) * 16 : 0;
        const int nr = wave_rows ? max(0, min(16, ne - r0)) : ne;
        const int t = wave_rows ? (tid & 63) : tid, nt = wave_rows ? 64 : BLOCK_THREADS;
        // this wave's LDS row stores before its own loads of them (other lanes' bytes)
        if (wave_rows) __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        const int nb16 = (nr * FROW) >> 4;
        const uint4 *src = reinterpret_cast<const uint4 *>(s_stk + r0 * FROW);
        uint4 *dst = reinterpret_cast<uint4 *>(o.img + (e0 + r0) * (int64_t)FROW);
        for (int i = t; i < nb16; i += nt) dst[i] = src[i];
        const int rem = ((nr * FROW) >> 2) - (nb16 << 2);          // trailing dwords (partial block)
        if (t < rem)
            reinterpret_cast<uint32_t *>(dst + nb16)[t] = reinterpret_cast<const uint32_t *>(src + nb16)[t];
    } else if (fast) {
        // Block-relative output dword k needs old dwords k+36, k+37 (alignbyte by 3) while its
        // env column j = k mod 147 <= 109; dword 110 mixes old byte 587 with new bytes 0..2;
        // dwords >= 111 are new-frame dwords (the LDS frame row holds new byte b at byte 1+b).
        // The old dwords were loaded into registers in phase 1, before any store: in place, no hazard.
        const uint32_t *f32 = reinterpret_cast<const uint32_t *>(s_stk);
        uint4 *g128 = reinterpret_cast<uint4 *>(o.img + e0 * (int64_t)IMG);
        // block-uniform masks in SGPRs: the terminal branch below is scalar
        const unsigned long long dmask = wave_uniform64(s_dmask), tmask = wave_uniform64(s_tmask);
#pragma unroll
        for (int r = 0; r < MAXQ; r++) {
            const int q = r * BLOCK_THREADS + tid, k = 4 * q;
            const int e0q = k / DW, j0 = k - e0q * DW;
            if (q < nq) {
                // Branch-free: the 4 frame-row dwords are read together (one LDS round trip),
                // then each output dword is a select of old / mixed / new.
                const uint32_t src[5] = {qa[r].x, qa[r].y, qa[r].z, qa[r].w, qb[r]};
                uint32_t fv[4];
                int e = e0q, j = j0;
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    fv[t] = f32[e * (FROW / 4) + max(j - 110, 0)];
                    if (++j == DW) { j = 0; e++; }
                }
                e = e0q; j = j0;
                uint32_t w[4];
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    const bool dn = (dmask >> e) & 1ull;
                    const uint32_t old = dn ? 0u : __builtin_amdgcn_alignbyte(src[t + 1], src[t], 3);
                    const uint32_t mix = (fv[t] & 0xFFFFFF00u) | (dn ? 0u : (src[t] >> 24));
                    w[t] = j <= 109 ? old : (j == 110 ? mix : fv[t]);
                    if (++j == DW) { j = 0; e++; }
                }
                if (!(MGX_DIAG_SKIP & 2)) stk_store(g128 + q, make_uint4(w[0], w[1], w[2], w[3]));
            }
        }
        if (tmask) {                                 // terminal_observation: the older frames (rare)
#pragma unroll
            for (int r = 0; r < MAXQ; r++) {
                const int q = r * BLOCK_THREADS + tid, k = 4 * q;
                const int e0q = k / DW, j0 = k - e0q * DW;
                const unsigned long long qm = (3ull << e0q) & ((j0 >= DW - 3) ? ~0ull : (1ull << e0q));
                if (q < nq && (tmask & qm)) {
                    const uint32_t src[5] = {qa[r].x, qa[r].y, qa[r].z, qa[r].w, qb[r]};
                    int e = e0q, j = j0;
#pragma unroll
                    for (int t = 0; t < 4; t++) {
                        if ((tmask >> e) & 1ull) {
                            uint8_t *trow = o.t_img + (e0 + e) * (int64_t)IMG;
                            if (j <= 109) reinterpret_cast<uint32_t *>(trow)[j] = __builtin_amdgcn_alignbyte(src[t + 1], src[t], 3);
                            else if (j == 110) trow[4 * 110] = (uint8_t)(src[t] >> 24);   // old byte 587
                        }
                        if (++j == DW) { j = 0; e++; }
                    }
                }
            }
        }
        // tail dword (partial last block whose row count is not a multiple of 4): its old
        // dwords come from rows no other thread of this block writes before the barrier below
        if (limit != nq * 4) {
            uint32_t tv = 0;
            if (kt < limit) {
                const int e = kt / DW, j = kt - e * DW;
                const bool dn = s_done[e];
                const uint32_t o36 = tq36, o37 = tq37;
                if (j <= 109) tv = dn ? 0u : __builtin_amdgcn_alignbyte(o37, o36, 3);
                else if (j == 110) tv = (f32[e * (FROW / 4)] & 0xFFFFFF00u) | (dn ? 0u : (o36 >> 24));
                else tv = f32[e * (FROW / 4) + (j - 110)];
                if (s_term[e]) {
                    uint8_t *trow = o.t_img + (e0 + e) * (int64_t)IMG;
                    if (j <= 109) reinterpret_cast<uint32_t *>(trow)[j] = __builtin_amdgcn_alignbyte(o37, o36, 3);
                    else if (j == 110) trow[4 * 110] = (uint8_t)(o36 >> 24);
                }
            }
            sync_lds();
            if (kt < limit) reinterpret_cast<uint32_t *>(o.img + e0 * (int64_t)IMG)[kt] = tv;
        }
    } else {
        uint8_t *gimg = o.img + e0 * (int64_t)IMG;
        const int NEWEST = IMG - FRAME;
        const int nbytes = ne * IMG;
        for (int b = tid; b < nbytes; b += BLOCK_THREADS) {
            const int e = b / IMG, off = b - e * IMG;
            int src = off + FRAME;
            if (src >= IMG) src -= IMG;
            gimg[b] = (s_done[e] && off < NEWEST) ? 0 : s_stk[e * IMG + src];
        }
    }

#if MGX_STAMPS
    tsC = __builtin_amdgcn_s_memtime();
#endif
    if (tid == 0) {
        // workgroup-private stats slot: fire-and-forget adds (no load on the kernel's tail)
        atomicAdd(&p.blk[blockIdx.x].x, (unsigned long long)ne);
        if (nd) atomicAdd(&p.blk[blockIdx.x].y, (unsigned long long)nd);
        if (s_ll) atomicAdd(&p.blk[blockIdx.x].z, s_ll);
#if MGX_STAMPS
        const unsigned long long ts4 = __builtin_amdgcn_s_memtime();
        atomicAdd(&p.counters[4], ts1 - ts0);   // phase 1: loads
        atomicAdd(&p.counters[5], tsA - ts1);   // phase 2a: step logic
#if MGX_STAMPS == 2
        atomicAdd(&p.counters[6], tsB - tsA);   // phase 2b: render
        atomicAdd(&p.counters[7], ts4 - ts2);   // phase 3+5: stack roll + grid write-back
#elif MGX_STAMPS == 3
        atomicAdd(&p.counters[6], tsC - ts2);   // phase 3: roll pass 2
        atomicAdd(&p.counters[7], ts4 - tsC);   // phase 5: grid write-back, ring heads, stats
#else
        atomicAdd(&p.counters[6], ts2 - tsA);   // phase 2b+2c: render, done envs, ring pops, render
        atomicAdd(&p.counters[7], ts4 - ts2);   // phase 3+5: stack roll + grid write-back
#endif
#endif
    }
    if (p.clk.slots) {                            // every wave of the workgroup is done
        __syncthreads();
        if (tid == 0) clk_record(p.clk, CLK_STEP, s_t0);
    }
}

// ======================================================= fused rollout kernel
// mgx_rollout_compact: K consecutive compact steps -- mgx_step_compact's transition, RNG streams,
// auto-resets and outputs, bit for bit -- of 64 envs per workgroup in ONE launch, for a rollout
// whose actions are known up front (a random-action or scripted rollout: BASELINE config 2's
// workload).  The per-step kernel is bound by latency, not bytes: its 1,024 workgroups all start
// together, so all of them wait on the same two load round trips (state, then the popped episode),
// then compute, then store, in lock-step.  Here the env state stays in registers and
// LDS between steps: a step loads nothing it must wait for -- its actions and the episodes it may
// pop are prefetched a step ahead by a fifth, DMA-only wave -- and the workgroups drift apart, so
// one's stores drain under another's step logic and render.
//   waves 0-3  as mgx_step_kernel<., true>: wave 0 = one lane per env (env_step), then all four
//              render 4 threads per env and copy their 16 rows out
//   wave 4     LDS-DMA only: actions of step t+1; for an env that popped at step t-1, its ring
//              episode after next, and the popped episode's RNG snapshot -> cur_rng (a step late:
//              only the MT slider reads it during the launch, and an older cursor is a lower bound).
//              Every env keeps its next TWO ring episodes staged (buffer = ring position & 1), so a
//              pop never waits.
// LDS: 4 workgroups + 4 refill waves per CU at S = 8 (26 + 13 KB each): the refill runs
// beside the whole launch instead of waiting for its workgroups to retire.
// Outputs of step t go to row t of [K][N] arrays; the env state, ring head and grids are written
// back once, at the end.  The refill may run concurrently (it reads ring_head once, at its start:
// a stale head only under-estimates its free slots); the K steps lie within one refill epoch, whose
// join published >= K episodes per env, so every staged slot is in [head, pub).
// ---- the synthetic random policy's draws (mgx_random_actions, mgx_set_random_policy; include/mgx.h): action i of
// launch c = Lemire's multiply-shift of the high half of splitmix64(key_c ^ i * M), key_c = splitmix64(seed + c * G)
__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t rnd_key(uint64_t seed, unsigned long long c) {
    return splitmix64(seed + (uint64_t)c * 0x9E3779B97F4A7C15ull);
}
__device__ __forceinline__ int32_t rnd_draw(uint64_t key, uint64_t i, uint32_t n_actions) {
    const uint64_t h = splitmix64(key ^ (i * 0xD1B54A32D192ED03ull));
    return (int32_t)(((h >> 32) * (uint64_t)n_actions) >> 32);
}

struct ROut {
    uint8_t *rows, *mids, *t_rows;   // [K][N][148], [K][N], [N][148]
    float *reward;                   // [K][N]
    double *reward64;                // [K][N] (optional)
    uint8_t *term, *trunc, *done;    // [K][N]
    float *ep_ret;                   // [N] as after the last step (optional)
    int32_t *ep_len, *livelock;      // [N] as after the last step (optional)
    // mgx_rollout_compact_gae: GAE of the launch's K steps in the epilogue (gadv null: none)
    const float *gv, *glv;           // values [K][N], last values [N]
    float gg, gc;                    // gamma, float(gamma * lambda)
    float *gadv, *gret;              // [K][N]
    double *gshard;                  // (sum A, sum A^2) partials (GAE_SHARDS x 2), or null
};
constexpr int ROLL_THREADS = BLOCK_THREADS + 64;


// Template flags keep what a config does not use out of the step loop (round 4: the loop held ~100 uniform
// values -- output pointers, feature flags, LDS bases -- and spilled 65 SGPRs to VGPR lanes, ~86 v_readlane per
// step): VIS see_through_walls == False (Grid.process_vis), MOVE 'move' missions (problems mov / full: target
// ranges), R64 the optional f64 rewards.  ep_return / ep_len / livelock (after the last step only) are kept in
// LDS and written after the loop.
// EPB: envs per block, 64 or 32 (round 5, S = 16: config 5's 63-KB workgroups fitted two to a CU; at 32 envs the
// same LDS per env, twice as many workgroups): 4 * EPB render threads (wave 0 also runs the step logic, lanes
// >= EPB idle) + the DMA wave.
template <bool VIS, bool MOVE, bool R64, int SC = 0, int EPB = BLOCK_ENVS>   // SC > 0: the grid size as a constant
__global__ __launch_bounds__(4 * EPB + 64, 4) void mgx_rollout_kernel(KParams p, ROut o, const int32_t *__restrict__ actions,
                                                                      int K) {
    static_assert(EPB == 64 || EPB == 32, "envs per block");
    constexpr int RT = 4 * EPB, RTH = RT + 64;       // render threads, all threads
    extern __shared__ __align__(16) uint8_t smem[];
    constexpr int CSTK = (EPB * FROW + 15) & ~15;
    const int GSQ = SC > 0 ? ((SC * SC + 15) & ~15) >> 4 : p.GS >> 4, GB = GSQ * EPB * 16;
    uint8_t *s_stk = smem;                                             // frame rows [64][148]
    uint8_t *s_grid = smem + CSTK;                                     // current grids (chunk-major, cm_off)
    uint8_t *s_pg = s_grid + GB;                                       // [2] staged ring episodes' grids
    uint4 *s_ph = reinterpret_cast<uint4 *>(s_pg + 2 * GB);            // [2][64] their headers
    int32_t *s_act = reinterpret_cast<int32_t *>(s_ph + 2 * EPB);   // [2][64] actions
    unsigned long long *s_mr = reinterpret_cast<unsigned long long *>(s_act + 2 * EPB);
                                                                       // [64] 'move' target_range (has_move only)
    __shared__ uint32_t s_rp[EPB];        // render params of the frame written (post-step view or
                                                 // the popped episode's first)
    __shared__ uint32_t s_rpt[EPB];       // post-step view of a finished episode (terminal row)
    __shared__ uint8_t s_term[EPB];       // terminal row written this step
    __shared__ uint8_t s_popb[EPB];       // staged buffer popped this step (0xFF: none)
    // [step & 1] new ring head of an env that popped; NO_POP: none (u32: every rpos_t value is a real one)
    __shared__ uint32_t s_nh[2][EPB];
    __shared__ unsigned long long s_tmask;
    // per-env state between steps lives in LDS, not registers: a loop-carried value would stay live
    // through the render, where the register pressure peaks (in registers: 128 VGPRs, 3 workgroups
    // per CU instead of 4)
    __shared__ uint4 s_st[EPB];           // EnvState
    __shared__ rpos_t s_head[EPB], s_pub[EPB];
    __shared__ unsigned long long s_cnt[2];      // resets, abandoned attempts
    __shared__ uint32_t s_err;
    __shared__ float s_lrew[EPB];         // the last step's reward, step count, abandoned attempts
    __shared__ int s_lsc[EPB], s_lll[EPB];

    const int tid = threadIdx.x, lane = tid & 63;     // (wave 0 and the DMA wave: env = lane, lanes >= EPB idle)
    const int64_t e0 = (int64_t)blockIdx.x * EPB;
    const int64_t N = p.n;
    const int ne = (int)min<int64_t>(EPB, N - e0);
    const int S = SC > 0 ? SC : p.S, D = p.D;
    const bool wave0 = tid < 64, dmaw = tid >= RT;
    const int lc = min(lane, ne - 1);
    __shared__ unsigned long long s_t0;           // kernel clock: this workgroup's start
    if (p.clk.slots && tid == 0) s_t0 = clk_now();
    // ---- setup: ring positions and state (waves 0 and 4), grids (waves 0-3, LDS-DMA)
    if (wave0 && lane < EPB) {
        s_st[lane] = reinterpret_cast<const uint4 *>(p.state)[e0 + lc];
        s_head[lane] = p.ring_head[e0 + lc];
        if (MOVE) s_mr[lane] = p.range_cur[e0 + lc];
        s_nh[1][lane] = NO_POP;
        if (lane < 2) s_cnt[lane] = 0;
        if (lane == 0) s_err = 0;
    }
    if (!dmaw && lane < EPB) {                       // (LDS-DMA: lane l writes chunk byte l * 16)
        const uint4 *src = reinterpret_cast<const uint4 *>(p.grid + (e0 + lc) * p.GS);
        for (int c = tid >> 6; c < GSQ; c += RT / 64)
            __builtin_amdgcn_global_load_lds(src + c, s_grid + c * (EPB * 16), 16, 0, 0);
    }
    // stage ring episode h of env e (this lane's) into buffer h & 1: header, grid
    auto stage = [&](rpos_t h) {
        const uint32_t slot = (uint32_t)(e0 + lane) * (uint32_t)D + (h & (D - 1));   // N * D < 2^32
        // the record's byte offset is 64-bit: N * D * REC reaches 2^33 at config 5 (131,072 x 256 x 320)
        const uint4 *gs = reinterpret_cast<const uint4 *>(
            p.ring_rec + (size_t)slot * (size_t)(SC > 0 ? (((GSQ << 4) + 48 + 63) & ~63) : p.REC));
        const uint4 *hs = gs + GSQ;
        // LDS-DMA destinations (M0) must be wave-uniform: one pass per buffer, each under the exec mask of
        // its lanes, as two separate branches -- NOT if / else.  From an if / else whose arms issue the same
        // loads to different LDS bases, the compiler sank a common load (chunk 3 at S = 8, the loop unrolled)
        // below the join and took its M0 from the first lane's arm (v_readfirstlane): the other parity's
        // lanes wrote that chunk into the wrong buffer (round 4).  The asm barriers keep each pass's loads in
        // its own branch.
        const uint32_t par = h & 1;
        if (par == 0) {
            __builtin_amdgcn_global_load_lds(hs, s_ph, 16, 0, 0);
            for (int c = 0; c < GSQ; c++) __builtin_amdgcn_global_load_lds(gs + c, s_pg + c * (EPB * 16), 16, 0, 0);
            asm volatile("" ::: "memory");
        }
        if (par != 0) {
            __builtin_amdgcn_global_load_lds(hs, s_ph + EPB, 16, 0, 0);
            for (int c = 0; c < GSQ; c++) __builtin_amdgcn_global_load_lds(gs + c, s_pg + GB + c * (EPB * 16), 16, 0, 0);
            asm volatile("" ::: "memory");
        }
    };
    rpos_t head0 = 0;                                // the DMA wave: this env's ring head at the launch's start
    // random policy (no actions buffer, mgx_set_random_policy): the DMA wave draws step t's actions itself, the
    // draws of mgx_random_actions over a [K][N] buffer at this launch's counter (the workgroup's own: every
    // workgroup runs every launch, so all of them hold the same count)
    const bool rnd = actions == nullptr;
    uint64_t rkey = 0;
    unsigned long long rc = 0;
    if (rnd && dmaw) {
        rc = *reinterpret_cast<volatile const unsigned long long *>(p.rnd_ctr + blockIdx.x);
        rkey = rnd_key(p.rnd_seed, rc);
    }
    if (dmaw && lane < ne) {
        if (rnd) s_act[lane] = rnd_draw(rkey, (uint64_t)(e0 + lane), 7u);
        else __builtin_amdgcn_global_load_lds(actions + e0 + lane, s_act, 4, 0, 0);
        // the end of the env's published episodes: ring_pubn, read ONCE (the slide after a refill running
        // beside this launch may raise it meanwhile; every value it takes is a completed refill's), shared
        // with the step wave through s_pub so that the staging and the pops agree
        // Visibility of the slots below the value read: every value ring_pubn takes is the tail of a refill
        // that has COMPLETED (the slide that writes it follows the refill on the refill stream, and a kernel's
        // stores are released at its end).  The load is an agent-scope ACQUIRE (ADVICE r3 / VERDICT r4): it
        // pairs with that release, and the cache invalidate it implies orders every later load of the slots
        // (LDS-DMA included) after it, whatever the slot lines' history in this CU's caches.  Once per env per
        // launch.
        const rpos_t rhead = p.ring_head[e0 + lane];
        const rpos_t rpub = __hip_atomic_load(p.ring_pubn + e0 + lane, MGX_PUBN_ACQUIRE ? __ATOMIC_ACQUIRE : __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
        head0 = rhead;
        s_pub[lane] = rpub;
        const int q = (rpos_t)(rpub - rhead);
        if (q > 0) stage(rhead);
        if (q > 1) stage((rpos_t)(rhead + 1));
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();

#if MGX_RSTAMPS
    // diagnostics (-DMGX_RSTAMPS): wave 0's clocks per phase, summed over the steps -> counters[4..7]
    unsigned long long rs_c[4] = {0, 0, 0, 0}, rs_t = 0;
#define RSTAMP(k) do { if (tid == 0) { const unsigned long long _t = __builtin_amdgcn_s_memtime(); \
                                       rs_c[(k) > 0 ? (k) - 1 : 0] += (k) > 0 ? _t - rs_t : 0ull; rs_t = _t; } } while (0)
#else
#define RSTAMP(k) do { } while (0)
#endif
    if (dmaw) {
        // ---- the DMA wave's own loop (round 4: the waves' loops are separate, so that the values only one
        // of them uses are not live across the other's: the single loop spilled 56-65 SGPRs).  Its barriers
        // match the compute waves' one for one: A, the terminal-row barriers when s_tmask (block-uniform),
        // process_vis's two, B.
        for (int t = 0; t < K; t++) {
            const int tb = t & 1;
            int tidv = tid;
            asm volatile("" : "+v"(tidv));
            const int lanev = tidv & 63;
            // the next step's actions; the ring episode after next of every env that popped last step
            // (LDS-DMA only: a register load here would make the wave wait for it -- and for every
            // prefetch in flight -- before the post-logic barrier, the whole block with it)
            if (lanev < ne) {
                if (t + 1 < K) {
                    if (rnd)
                        s_act[(tb ^ 1) * EPB + lanev] = rnd_draw(rkey, (uint64_t)(t + 1) * (uint64_t)N + (uint64_t)(e0 + lanev), 7u);
                    else
                        __builtin_amdgcn_global_load_lds(actions + (int64_t)(t + 1) * N + e0 + lanev,
                                                         s_act + (tb ^ 1) * EPB, 4, 0, 0);
                }
                const uint32_t nh = s_nh[tb ^ 1][lanev];
                if (nh != NO_POP && (rpos_t)(s_pub[lanev] - nh) > 1) stage((rpos_t)(nh + 1));
            }
            // A: its loads (next step's actions and episodes) need not have landed yet
            if (MGX_ROLL_VMKEEP >= 0) sync_keep_vm<63>(); else __syncthreads();
            if (s_tmask) {
                __syncthreads();
                if (VIS) __syncthreads();
                __syncthreads();
                __syncthreads();
            }
            if (VIS) {
                __syncthreads();
                __syncthreads();
            }
            __builtin_amdgcn_s_waitcnt(0);                     // this step's prefetches have landed ...
            __syncthreads();                                   // B: ... before the next step reads them
        }
    } else {
        // Step t's frame rows are copied out by waves 1-3 during step t + 1's logic (wave 0
        // alone), before its post-logic barrier, instead of by every wave at the end of step t: the copy-out
        // leaves the step's critical path (the last step's rows after the loop).  s_stk is rewritten only after
        // that barrier (terminal rows, render).
        const auto rows_out_block = [&](int t_rows, int tt, int nt) {
            const int nb16 = (ne * FROW) >> 4;
            const uint4 *src = reinterpret_cast<const uint4 *>(s_stk);
            uint4 *dst = reinterpret_cast<uint4 *>(o.rows + ((int64_t)t_rows * N + e0) * FROW);
            for (int i = tt; i < nb16; i += nt) st16<MGX_NT_ROWS != 0>(dst + i, src[i]);
            const int rem = ((ne * FROW) >> 2) - (nb16 << 2);
            if (tt < rem)
                reinterpret_cast<uint32_t *>(dst + nb16)[tt] = reinterpret_cast<const uint32_t *>(src + nb16)[tt];
        };
        unsigned long long nres = 0;                 // wave 0: resets so far (ballot popcounts; s_cnt[0] after the loop)
        for (int t = 0; t < K; t++) {
            const int tb = t & 1;
            RSTAMP(0);
            if (t > 0 && !wave0) {
                int tq = tid;
                asm volatile("" : "+v"(tq));
                rows_out_block(t - 1, tq - 64, RT - 64);
            }
            // thread index through an opaque copy: lane- / env-derived addresses are then computed inside
            // each region of the step, instead of being hoisted out of the loop and kept live through all of
            // them (96 -> fewer VGPRs; the render's and the step logic's registers no longer add up)
            int tidv = tid;
            asm volatile("" : "+v"(tidv));
            const int lanev = tidv & 63;
            if (wave0) {
                // ---- the step: one lanev per env.  The block waits for this one wave at the post-logic barrier:
                // MGX_ROLL_LOGIC_PRIO raises its issue priority for the phase (over the co-resident refill waves'
                // priority 2), back to 0 for the render
                if (MGX_ROLL_LOGIC_PRIO == 3) __builtin_amdgcn_s_setprio(3);
                else if (MGX_ROLL_LOGIC_PRIO == 2) __builtin_amdgcn_s_setprio(2);
                else if (MGX_ROLL_LOGIC_PRIO == 1) __builtin_amdgcn_s_setprio(1);
                bool tw = false;
                uint8_t popb = 0xFF;
                uint32_t nh = NO_POP;
                if (lanev < ne) {
                    const uint32_t e = (uint32_t)(e0 + lanev), oi = (uint32_t)t * (uint32_t)N + e;   // N * K < 2^32
                    EnvState st;
                    {
                        const uint4 sv = s_st[lanev];
                        __builtin_memcpy(&st, &sv, sizeof st);
                    }
                    rpos_t rhead = s_head[lanev];
                    uint64_t mrange = MOVE ? s_mr[lanev] : 0ull;
                    uint32_t err = 0;
                    int a = s_act[tb * EPB + lanev];
                    // every LDS read the step may need, issued together with the state's (round 5): the published
                    // end and BOTH staged headers (the popped buffer is rhead & 1, known only after s_head lands) --
                    // the pop no longer waits on two more dependent LDS round trips after the step logic
                    const rpos_t rpub = s_pub[lanev];
                    const uint4 h0 = s_ph[lanev], h1 = s_ph[EPB + lanev];
                    if ((unsigned)a > 6u) { err |= MGX_DEVERR_BAD_ACTION; a = -1; }
                    const StepRes r = env_step<EPB>(st, a, s_grid, lanev, S, p.manual, mrange);
                    tw = r.done && (p.terminal_mode == MGX_TERMINAL_ALL ||
                                    (p.terminal_mode == MGX_TERMINAL_TRUNCATED && r.trunc && !r.term));
                    s_rpt[lanev] = r.view;
                    o.reward[oi] = (float)r.rew;
                    if (R64) o.reward64[oi] = r.rew;
                    o.term[oi] = r.term;
                    o.trunc[oi] = r.trunc;
                    o.done[oi] = r.done;
                    if (t == K - 1) {                        // written out after the loop
                        s_lrew[lanev] = (float)r.rew;        // (only the final step can pay a reward)
                        s_lsc[lanev] = r.sc;
                    }
                    uint8_t mid = st.mission_id;
                    int lvl = 0;
                    if (r.done && (rpos_t)(rpub - rhead) != 0) {
                        // SubprocVecEnv auto-reset: the staged ring episode (header, RNG snapshot, grid)
                        popb = rhead & 1;
                        const uint4 h = popb ? h1 : h0;
                        if (MOVE) s_mr[lanev] = p.ring_range[e * (uint32_t)D + (rhead & (D - 1))];
                        mid = (uint8_t)(h.y >> 16);
                        st.ax = (uint8_t)(h.x & 0xFF); st.ay = (uint8_t)((h.x >> 8) & 0xFF); st.dir = (uint8_t)((h.x >> 16) & 0xFF);
                        st.carry = 0; st.step_count = 0; st.reward_step = (int16_t)r.rs;     // survives the reset (Q2)
                        st.tx = (uint8_t)(h.x >> 24); st.ty = (uint8_t)h.y; st.target_action = (uint8_t)(h.y >> 8);
                        st.mission_id = mid; st.mission_done = (uint8_t)r.mdone; st.frames = 1; st.flags = 0; st.pad = 0;
                        s_rp[lanev] = h.x & 0xFFFFFFu;
                        rhead++;
                        s_head[lanev] = rhead;
                        nh = rhead;
                        if (h.z) atomicAdd(&s_cnt[1], (unsigned long long)h.z);
                        lvl = (int)h.z;
                    } else {
                        if (r.done) err |= MGX_DEVERR_RING_EMPTY;   // cannot happen (refill production rule)
                        st.ax = (uint8_t)(r.view & 0xFF); st.ay = (uint8_t)((r.view >> 8) & 0xFF);
                        st.dir = (uint8_t)((r.view >> 16) & 3); st.carry = r.carry;
                        st.step_count = (uint16_t)r.sc; st.reward_step = (int16_t)r.rs; st.mission_done = (uint8_t)r.mdone;
                        s_rp[lanev] = r.view;
                    }
                    o.mids[oi] = mid;
                    if (t == K - 1) s_lll[lanev] = lvl;
                    {
                        uint4 sv;
                        __builtin_memcpy(&sv, &st, sizeof st);
                        s_st[lanev] = sv;
                    }
                    if (err) atomicOr(&s_err, err);
                }
                if (lanev < EPB) {
                    s_term[lanev] = tw;
                    s_popb[lanev] = popb;
                    s_nh[tb][lanev] = nh;
                }
                const unsigned long long tm = __ballot(tw);
                // resets: one popcount of the wave's pops, added by lane 0 (only wave 0 writes s_cnt), instead of
                // a 64-bit LDS atomic per popping lane on one address (round 4)
                const unsigned long long pm = __ballot(popb != 0xFF);
                nres += (unsigned long long)__popcll(pm);   // (wave-uniform: a scalar register, written after the loop)
                if (lanev == 0) s_tmask = tm;
                if (MGX_ROLL_LOGIC_PRIO) __builtin_amdgcn_s_setprio(0);
            }
            RSTAMP(1);                                     // step logic (wave 0)
            sync_keep_vm<MGX_ROLL_VMKEEP>();
            RSTAMP(2);                                     // wait for the block
            // (every barrier below is matched by the DMA wave's loop)
            const int le = tidv >> 2, q = tidv & 3;
            if (s_tmask) {
                // terminal rows (rare, block-uniform): the finished episode's last view, rendered into the
                // env's frame row from its post-step grid and copied out before the row is reused below
                if (le < ne && s_term[le]) {
                    if (VIS) render_cols<EPB>(s_grid, S, le, q, s_rpt[le], s_stk + le * FROW + 1);
                    else render_row<EPB>(s_grid, S, le, q, s_rpt[le], s_stk + le * FROW);
                }
                __syncthreads();
                if (VIS) {
                    if (tidv < ne && s_term[tidv]) apply_vis(s_stk + tidv * FROW + 1);
                    __syncthreads();
                }
                if (tidv < ne && s_term[tidv]) s_stk[tidv * FROW] = (uint8_t)((s_rpt[tidv] >> 16) & 3);
                __syncthreads();
                if (le < ne && s_term[le]) {
                    const uint32_t *fr = reinterpret_cast<const uint32_t *>(s_stk + le * FROW);
                    uint32_t *tr = reinterpret_cast<uint32_t *>(o.t_rows + (e0 + le) * (int64_t)FROW);
    #pragma unroll 1
                    for (int k = 10 * q; k < min(10 * q + 10, FROW / 4); k++) tr[k] = fr[k];
                }
                __syncthreads();
            }
            // the frame of every env: the new episode's first where one was popped (rendered straight from
            // its staged grid, which then becomes the env's grid)
            if (le < ne) {
                const uint8_t b = s_popb[le];
                const uint8_t *g = b == 0xFF ? s_grid : s_pg + b * GB;
                const uint32_t rp = s_rp[le];
                if (VIS) {
                    render_cols<EPB>(g, S, le, q, rp, s_stk + le * FROW + 1);
                    if (q == 0) s_stk[le * FROW] = (uint8_t)((rp >> 16) & 3);
                } else {
                    render_row<EPB>(g, S, le, q, rp, s_stk + le * FROW);
                }
                if (b != 0xFF)
                    for (int c = q; c < GSQ; c += 4)
                        *reinterpret_cast<uint4 *>(s_grid + c * (EPB * 16) + le * 16) =
                            *reinterpret_cast<const uint4 *>(g + c * (EPB * 16) + le * 16);
            }
            if (VIS) {
                __syncthreads();
                if (tidv < ne) apply_vis(s_stk + tidv * FROW + 1);
                __syncthreads();
            }
            RSTAMP(3);                                     // terminal rows + render
            sync_keep_vm<MGX_ROLL_VMKEEP>();               // B
            RSTAMP(4);                                     // rows out + the block barrier
        }
        if (K > 0) rows_out_block(K - 1, tid, RT);   // the last step's rows
        if (wave0 && lane == 0) s_cnt[0] = nres;     // (read after the write-back section's barrier)
    }
    if (o.gadv) {
        // mgx_rollout_compact_gae: mgx_gae_kernel<true>'s recurrence (same fp32 op order) for this workgroup's envs
        // over the K steps it just ran.  Round 5: the rewards / dones it wrote and the caller's values are staged in
        // LDS tiles of GAE_RT steps by all five waves -- one load round trip per tile -- in the frame-row area,
        // free once the last rows are out; wave 0 then runs the recurrence from LDS (round 4: wave 0 alone read
        // them back in dependent batches of 8 steps, ~15 us on the launch's tail).
        constexpr int GAE_RT = 16;                       // [16][64] f32 r, f32 v, u8 d = 9,216 B <= the 9,472-B rows
        static_assert(GAE_RT * EPB * 9 <= ((EPB * FROW + 15) & ~15), "GAE tile in the frame rows");
        float *g_r = reinterpret_cast<float *>(s_stk), *g_v = g_r + GAE_RT * EPB;
        uint8_t *g_d = reinterpret_cast<uint8_t *>(g_v + GAE_RT * EPB);
        __syncthreads();                                 // the last rows' copy-out has read s_stk
        const bool act = wave0 && lane < ne;
        float last = 0.0f, nv = act ? o.glv[e0 + lane] : 0.0f;
        double s1 = 0.0, s2 = 0.0;
        for (int thi = K - 1; thi >= 0; thi -= GAE_RT) {
            const int nt = min(GAE_RT, thi + 1);
            for (int idx = tid; idx < nt * EPB; idx += RTH) {
                const int i = idx / EPB, l = idx & (EPB - 1);
                if (l < ne) {
                    const int64_t k = (int64_t)(thi - i) * N + e0 + l;
                    g_r[idx] = o.reward[k];
                    g_v[idx] = o.gv[k];
                    g_d[idx] = o.done[k];
                }
            }
            __syncthreads();
            if (act) {
                for (int i = 0; i < nt; i++) {
                    const int64_t k = (int64_t)(thi - i) * N + e0 + lane;
                    const float rr = g_r[i * EPB + lane], vv = g_v[i * EPB + lane];
                    const float nnt = 1.0f - (float)g_d[i * EPB + lane];
                    const float delta = (rr + (o.gg * nv) * nnt) - vv;
                    last = delta + (o.gc * nnt) * last;
                    o.gadv[k] = last;
                    o.gret[k] = last + vv;
                    s1 += (double)last;
                    s2 += (double)last * (double)last;
                    nv = vv;
                }
            }
            __syncthreads();                             // wave 0 has read the tile before the next one lands
        }
        if (o.gshard && wave0) {
            for (int off = 32; off > 0; off >>= 1) {
                s1 += __shfl_down(s1, off);
                s2 += __shfl_down(s2, off);
            }
            if (lane == 0) {
                double *sh = o.gshard + 2 * (blockIdx.x & 255);   // GAE_SHARDS slots, as mgx_gae_kernel
                atomicAdd(&sh[0], s1);
                atomicAdd(&sh[1], s2);
            }
        }
    }
#if MGX_RSTAMPS
    if (tid == 0)
        for (int k = 0; k < 4; k++) atomicAdd(&p.counters[4 + k], rs_c[k]);
#endif
#undef RSTAMP
    // ---- write back: state and ring head (wave 0), every grid, counters; the DMA wave: cur_rng of
    // the envs that popped at the last step
    // cur_rng of every env that popped in this launch: the RNG snapshot of its last pop, once, at the end
    // (round 3: copied a step after every pop, the DMA wave's register loads made it wait before the
    // post-logic barrier).  Meanwhile only the MT slider reads cur_rng, and an older cursor is a lower
    // bound of the live ones.
    // The snapshot is LOADED before the new head is published (a barrier between them): once ring_head
    // moves, a refill running beside this launch may reuse that slot (the head store raced the
    // load).  Stored to cur_rng after the barrier.
    uint4 rng0 = make_uint4(0, 0, 0, 0), rng1 = rng0;
    const bool rng_w = dmaw && lane < ne && s_head[lane] != head0;
    if (rng_w) {
        const uint32_t slot = (uint32_t)(e0 + lane) * (uint32_t)D + ((rpos_t)(s_head[lane] - 1) & (D - 1));
        const uint4 *rec = reinterpret_cast<const uint4 *>(
            p.ring_rec + (size_t)slot * (size_t)(SC > 0 ? (((GSQ << 4) + 48 + 63) & ~63) : p.REC));
        rng0 = rec[GSQ + 1];
        rng1 = rec[GSQ + 2];
    }
    if (dmaw) __builtin_amdgcn_s_waitcnt(0);         // the loads have returned ...
    __syncthreads();                                 // ... before wave 0 stores the heads below
    if (rng_w) {
        p.cur_rng[2 * (e0 + lane)] = rng0;
        p.cur_rng[2 * (e0 + lane) + 1] = rng1;
    }
    if (wave0 && lane < ne) {
        reinterpret_cast<uint4 *>(p.state)[e0 + lane] = s_st[lane];
        p.ring_head[e0 + lane] = s_head[lane];
        if (MOVE) p.range_cur[e0 + lane] = s_mr[lane];
        if (o.ep_ret) o.ep_ret[e0 + lane] = s_lrew[lane];
        if (o.ep_len) o.ep_len[e0 + lane] = s_lsc[lane];
        if (o.livelock) o.livelock[e0 + lane] = s_lll[lane];
    }
    if (!dmaw) {
        uint4 *dst = reinterpret_cast<uint4 *>(p.grid + e0 * p.GS);
        for (int i = tid; i < ne * GSQ; i += RT) {
            const int le = i / GSQ, c = i - le * GSQ;
            dst[i] = *reinterpret_cast<const uint4 *>(s_grid + c * (EPB * 16) + le * 16);
        }
    }
    if (rnd && tid == RT) p.rnd_ctr[blockIdx.x] = rc + 1ull;   // (a lane of the DMA wave: a vector store)
    if (tid == 0) {
        const int sb = (int)(blockIdx.x / (64 / EPB));   // the stats slot of these 64 envs (32-env blocks: two)
        atomicAdd(&p.blk[sb].x, (unsigned long long)ne * (unsigned long long)K);
        if (s_cnt[0]) atomicAdd(&p.blk[sb].y, s_cnt[0]);
        if (s_cnt[1]) atomicAdd(&p.blk[sb].z, s_cnt[1]);
        if (s_err) atomicOr(p.err, s_err);
    }
    if (p.clk.slots) {                            // every wave of the workgroup is done
        __syncthreads();
        if (tid == 0) clk_record(p.clk, EPB == 32 ? CLK_ROLL32 : CLK_STEP, s_t0);
    }
}

// ============================================================== fixup kernel
// Generates, inline, the next episode of every env the step kernel found with an
// empty ring (normally none; every done env when the ring is disabled), and writes
// that env's reset outputs.  Grid-stride over the list; the last workgroup to
// finish clears the list for the next step.
template <int NW, bool EXT>
__global__ __launch_bounds__(64) void mgx_fixup_kernel(KParams p, KOut o) {
    extern __shared__ __align__(16) uint8_t smem[];
    const int tid = threadIdx.x;
    uint8_t *s_grid = smem;                                   // [64][GSL]
    uint8_t *s_scr = smem + ((64 * p.GSL + 15) & ~15);        // [64] windows + objs
    const uint32_t cnt = *reinterpret_cast<volatile uint32_t *>(p.fix_count);
    unsigned long long ll = 0, maxcur = 0;
    uint32_t err = 0;
    for (uint32_t idx = blockIdx.x * 64 + tid; idx < cnt; idx += gridDim.x * 64) {
        const int64_t e = p.fix_list[idx];
        Gen<NW> G;
        load_gen(G, p, e, s_grid + tid * p.GSL, s_scr, tid);
        load_rng(G, p, e);
        if (p.start_rng) rng_snapshot(G, p.start_rng + 2 * e);
        ResetOut R;
        reset_env<NW, EXT>(G, R);
        if (G.nobjs > p.obj_cap) G.err |= 8u;   // objs list ran past its per-config capacity
        store_rng(G, p, e);
        rng_snapshot(G, p.cur_rng + 2 * e);
        {
            uint4 *dst = reinterpret_cast<uint4 *>(p.grid + e * p.GS);
            for (int c = 0; c < (p.GS >> 4); c++) {
                const uint32_t *q = reinterpret_cast<const uint32_t *>(G.g + c * 16);
                dst[c] = make_uint4(q[0], q[1], q[2], q[3]);
            }
        }
        EnvState ns = p.state[e];                  // carries mission_done / stored reward (Q2)
        ns.ax = (uint8_t)G.ax; ns.ay = (uint8_t)G.ay; ns.dir = (uint8_t)G.adir; ns.carry = 0;
        ns.step_count = 0;
        ns.tx = R.tx; ns.ty = R.ty; ns.target_action = R.ta; ns.mission_id = R.mission_id;
        ns.frames = 1; ns.flags = 0; ns.pad = 0;
        p.state[e] = ns;
        if (p.has_move) p.range_cur[e] = R.range;
        write_fresh_frame(p, o.img, e, G.g, G.ax, G.ay, G.adir);   // older slots were zeroed by the step
        dir_stack_fresh(o.dir, e, p.n_stack, G.adir);
        write_mission_stack(o.mis, p.mission64, e, p.n_stack, 1, p.mtok + R.mission_id * 32);
        if (o.livelock) o.livelock[e] = R.livelocks;
        ll += (unsigned long long)R.livelocks;
        maxcur = G.cur > maxcur ? G.cur : maxcur;
        err |= G.err;
    }
    for (int off = 32; off > 0; off >>= 1) {
        ll += __shfl_down(ll, off);
        const unsigned long long m = __shfl_down(maxcur, off);
        maxcur = m > maxcur ? m : maxcur;
        err |= __shfl_down(err, off);
    }
    if (tid == 0 && cnt) {                                     // nothing listed: no bookkeeping at all
        ulonglong4 b = p.blk[p.nblk + blockIdx.x];
        b.z += ll; b.w = b.w > maxcur ? b.w : maxcur;
        p.blk[p.nblk + blockIdx.x] = b;
        if (err) atomicOr(p.err, err);
        __threadfence();
        if (atomicAdd(p.fix_done, 1u) == gridDim.x - 1) {   // every workgroup has read `cnt`
            *p.fix_count = 0;
            *p.fix_done = 0;
        }
    }
}

// ========================================================= prefix records
// The prefix of an attempt that starts at stream word `pos`, decoded straight from the packed ring (no LDS window):
// the generator's own prefix_draws over a register queue that reads groups from global memory.
struct PfxQ {
    const uint64_t *table;
    uint64_t rmask;
    uint64_t cur, astart, gi, ga, gb, gc;
    int go;
    uint32_t llw, err;
    bool abort;
#if MGX_GEN_STAMPS
    unsigned long long *stamps;
    uint64_t tlast;
#endif
};
__device__ __forceinline__ uint64_t win_group(PfxQ &Q, uint64_t g) { return Q.table[g & Q.rmask]; }
__device__ __forceinline__ uint64_t pfx_index(uint64_t pos, uint64_t rmask) {
    const uint64_t g = div10(pos);
    return (g & rmask) * MT_FIELDS + (pos - g * MT_FIELDS);
}
__device__ __forceinline__ uint32_t pfx_tag(uint64_t pos, int shift) { return (uint32_t)(div10(pos) >> shift) & 0xFFu; }
// the record for `pos` (0: none -- its prefix would read past the words generated, or takes > 255 of them)
__device__ __forceinline__ uint64_t pfx_compute(const KParams &p, uint64_t pos) {
#if MGX_GEN_STAMPS
    return 0;
#else
    PfxQ Q;
    Q.table = p.mt;
    Q.rmask = p.mt_mask;
    Q.cur = Q.astart = pos;
    const uint64_t g = div10(pos);
    Q.go = (int)(pos - g * MT_FIELDS);
    Q.gi = g;
    Q.ga = win_group(Q, g);
    Q.gb = win_group(Q, g + 1);
    Q.gc = win_group(Q, g + 2);
    Q.llw = p.llw;
    Q.err = 0;
    Q.abort = false;
    Prefix P;
    prefix_draws(Q, p.S, p.cfg_mission < 0, p.all_doors_open != 0, P);
    const uint64_t adv = Q.cur - pos;
    if (Q.abort || adv == 0 || adv > 255) return 0;
    return pfx_pack(P, (uint32_t)adv, pfx_tag(pos, p.mt_shift));
#endif
}
// records for positions [lo, hi) (mgx_create: the host-generated start of the stream)
__global__ __launch_bounds__(256) void mgx_prefix_kernel(KParams p, uint64_t lo, uint64_t hi) {
    for (uint64_t pos = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; pos < hi;
         pos += (uint64_t)gridDim.x * blockDim.x)
        p.pfx[pfx_index(pos, p.mt_mask)] = pfx_compute(p, pos);
}
constexpr int PFX_PER_THREAD = 2;   // records each slide thread computes per launch (4,096 threads at 65,536 envs)

// ============================================================= refill kernel
// Pre-generates each env's next episodes into its ring until it holds D.
// Generation is a long serial RNG chain per env (~10^4 dependent ops); doing
// it here, batched every `refill_every` steps for all envs at once, takes it
// off the step kernel's critical path.  Episodes are generated in exactly the
// order the env will consume them, so RNG streams advance as in the reference.
// One wave per workgroup; all LDS is lane-private (grid row + MT window + objs).
// EPW: envs per wave (64, or 32 with lanes 32-63 idle: twice the waves, each running the union of fewer
// lanes' paths -- for grids whose 64-env waves would leave SIMDs without a refill wave, config 4).
template <int NW, bool EXT, bool MULTI, int SC = 0, int EPW = 64>   // SC > 0: the grid size as a constant
__device__ __forceinline__ void refill_body(const KParams &p) {
    extern __shared__ __align__(16) uint8_t smem[];
    const int tid = threadIdx.x;
    const int64_t e = tid < EPW ? (int64_t)blockIdx.x * EPW + tid : INT64_MAX;   // idle lanes: e >= n
    uint8_t *s_grid = smem;                                   // [64][GSL]
    uint8_t *s_scr = smem + ((64 * p.GSL + 15) & ~15);        // [64] windows + objs
    unsigned long long maxcur = 0;
    uint32_t err = 0;
    // issue priority over co-resident step / rollout waves (MGX_REFILL_PRIO; wave-uniform)
    if (p.refill_prio == 1) __builtin_amdgcn_s_setprio(1);
    else if (p.refill_prio == 2) __builtin_amdgcn_s_setprio(2);
    else if (p.refill_prio == 3) __builtin_amdgcn_s_setprio(3);
    __shared__ unsigned long long s_t0;           // kernel clock: this wave's start
    if (p.clk.slots && tid == 0) s_t0 = clk_now();
#if MGX_REFILL_CLOCK
    const unsigned long long rc0 = __builtin_amdgcn_s_memtime();   // diagnostics: wave clocks per launch
    int rc_iters = 0;
#endif
    // The step kernel may be popping this env's ring concurrently: `head` can be stale
    // (older, smaller), which only under-estimates the free slots.
    rpos_t tail = 0;
    int level = 0, cons = 0;
    if (e < p.n) {
        const rpos_t head = *reinterpret_cast<volatile const rpos_t *>(p.ring_head + e);
        tail = p.ring_tail[e];
        level = (int)(rpos_t)(tail - head);
        cons = (int)(rpos_t)(head - p.ring_seen[e]);     // episodes popped since the last refill read
        p.ring_seen[e] = head;
    }
    const int space = p.D - level, need = 2 * p.K - level;
    // Production: at least what keeps >= K episodes queued at the next join (each step pops
    // <= 1, so 2K - level), plus up to `cap` more while there is room.  Capping the per-epoch
    // production balances work across the lanes of a wave (its time is the busiest lane's)
    // while rings with slack absorb bursts of short episodes.  The cap is the wave's mean CONSUMPTION
    // since the last refill, rounded up (round 3; a fixed cap must sit well above the mean, and a
    // mean-deficit cap settles above it too), so the wave runs about as many attempt rounds as its lanes
    // popped on average while the lanes that popped more keep a deficit the ring depth absorbs -- and at
    // most the grid-wide round cap (round 4, below).
    int cap = p.cap;
    if (cap > 0 && !p.initial_fill) {
        int sum = e < p.n ? cons : 0, cnt = e < p.n ? 1 : 0;
        for (int off = 32; off > 0; off >>= 1) {
            sum += __shfl_xor(sum, off);
            cnt += __shfl_xor(cnt, off);
        }
        cnt = max(cnt, 1);
        cap = (sum + cnt - 1) / cnt;
        // The launch lasts as long as its slowest wave, and a wave runs as many attempt rounds as its
        // cap: one ceiling common to all waves (mgx_mt_slide_kernel: the grid's mean consumption per env
        // plus a margin, in whole rounds whose average is that target) keeps the waves whose lanes
        // popped more than the rest from setting the launch.  Their lanes keep the difference as a
        // deficit, which the ring depth absorbs and later epochs pay back.
        const int rc = p.mtc->round_cap;                           // wave-uniform (scalar load)
        if (rc > 0) cap = min(cap, rc);
    }
    int nfree = 0, nmin = 0;
    if (e < p.n) {
        // mgx_reset's fill: every ring to D (not just the invariant's 2K), so the epochs that follow
        // start at steady state: production then tracks consumption at once instead of running
        // need-driven rounds until the rings have filled (1,500+ steps at a cap near consumption)
        nfree = p.initial_fill ? space : max(need, p.cap < 0 ? space : min(cap, space));
        nfree = min(nfree, space);
        nmin = max(need, 0);                       // what the ring invariant requires this epoch
    }
    const bool producer = nfree > 0;
    if (__ballot(producer)) {
        Gen<NW> G;
        load_gen(G, p, e, s_grid + tid * p.GSL, s_scr, tid);
        if (SC > 0) G.S = SC;                      // (p.S == SC: the host picks this kernel for it)
        int livelocks = 0;
        if (producer) {
            load_rng(G, p, e);
            livelocks = (int)(p.aux[e].y >> 1);    // abandoned attempts carried over from the last epoch
        }
        // The lane's objs list (dead once its attempt is done) stages the episode's header + RNG snapshot for
        // the wave's record write; its grid is already in LDS (G.g)
        uint32_t *const stg = G.objs;
        // prefix record of this lane's next attempt, loaded ahead: right after the attempt before it ends (its cursor
        // is final then), so the load flies during the round's record write
        uint64_t nrec = 0;
        if (producer && p.pfx) nrec = p.pfx[pfx_index(G.cur, p.mt_mask)];
        // One attempt per round for every lane: a lane whose attempt live-locked retries while the others
        // already generate their next episode, exactly reset_env's retry semantics per env.  `nfree` budgets
        // ATTEMPTS: an abandoned attempt costs the lane one episode of this epoch's production (unless the
        // invariant needs it), not the wave an extra round -- the retry then continues in the next epoch, its
        // count carried in aux.  The rounds are wave-uniform (the record write below needs every lane).
        while (__ballot(nfree > 0)) {
#if MGX_REFILL_CLOCK
            rc_iters += nfree > 0;
#endif
            bool wrote = false;
            uint32_t slot = 0;
            if (nfree > 0) {
                ResetOut R;
                G.astart = G.cur;
                G.abort = false;
                // a record of this position from the stream's current pass: its words are consumed here, gen_multi
                // takes its draws from it (the prefix never reaches the live-lock cap: <= 255 of llw words)
                G.phave = p.pfx && (nrec & 0xFFu) && ((uint32_t)(nrec >> 8) & 0xFFu) == pfx_tag(G.cur, p.mt_shift);
                G.prec = nrec;
                if (G.phave) G.cur += nrec & 0xFFu;
                mt_sync(G);
                gen_attempt<NW, EXT, MULTI>(G, R);
                if (p.pfx) nrec = p.pfx[pfx_index(G.cur, p.mt_mask)];
                if (G.nobjs > p.obj_cap) G.err |= 8u;
                if (G.abort && ++livelocks <= 100000) {
                    if (nfree > nmin) nfree--;
                } else {
                    if (G.abort) G.err |= 4u;       // give up on this env (reported, never silent)
                    R.livelocks = livelocks;
                    livelocks = 0;
                    nfree--;
                    nmin--;
                    slot = (uint32_t)e * (uint32_t)p.D + (tail & (p.D - 1));    // N * D < 2^32
                    const uint4 h = pack_hdr(G, R);
                    uint4 rs[2];
                    rng_snapshot(G, rs);
                    stg[0] = h.x; stg[1] = h.y; stg[2] = h.z; stg[3] = h.w;
                    stg[4] = rs[0].x; stg[5] = rs[0].y; stg[6] = rs[0].z; stg[7] = rs[0].w;
                    stg[8] = rs[1].x; stg[9] = rs[1].y; stg[10] = rs[1].z; stg[11] = rs[1].w;
                    if (EXT && p.has_move) p.ring_range[slot] = R.range;
                    tail++;
                    wrote = true;
                }
            }
            // The round's records, written by the whole wave: piece j (16 B) of lane src's record by lane
            // q % 64 of pass q / 64, q = src * P + j -- consecutive lanes store consecutive pieces, so every
            // record (REC = 128 B at S = 8: one line) is one coalesced write
            const unsigned long long wm = __ballot(wrote);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   // the lanes' LDS stages ...
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // ... before the other lanes read them
            const int REC = SC > 0 ? ((((SC * SC + 15) & ~15) + 48 + 63) & ~63) : p.REC;
            const int P = REC >> 4, GQ = (SC > 0 ? ((SC * SC + 15) & ~15) : p.GS) >> 4;
            const uint8_t *objs0 = reinterpret_cast<const uint8_t *>(stg) - tid * (p.obj_stride * 4);
            for (int q = tid; q < 64 * P; q += 64) {
                const int src = q / P, j = q - src * P;
                const uint32_t ss = (uint32_t)__shfl((int)slot, src);
                if (!((wm >> src) & 1ull)) continue;
                const uint32_t *w = j < GQ ? reinterpret_cast<const uint32_t *>(s_grid + src * p.GSL + 16 * j)
                                           : reinterpret_cast<const uint32_t *>(objs0 + src * (p.obj_stride * 4) +
                                                                                 16 * (j - GQ));
                uint4 v = make_uint4(0u, 0u, 0u, 0u);
                if (j < GQ + 3) v = make_uint4(w[0], w[1], w[2], w[3]);
                st16<MGX_NT_REC != 0>(reinterpret_cast<uint4 *>(p.ring_rec + (size_t)ss * (size_t)REC) + j, v);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   // (the next round rewrites the stages)
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        if (producer) {
            store_rng(G, p, e, (uint32_t)livelocks);
            p.ring_tail[e] = tail;                 // published by the slide that follows (ring_pubn)
            maxcur = G.cur;
            err = G.err;
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        unsigned long long o = __shfl_down(maxcur, off);
        maxcur = o > maxcur ? o : maxcur;
        err |= __shfl_down(err, off);
#if MGX_REFILL_CLOCK
        rc_iters = max(rc_iters, __shfl_down(rc_iters, off));
#endif
    }
#if MGX_REFILL_CLOCK
    if (tid == 0) {
        atomicAdd(&p.counters[26], __builtin_amdgcn_s_memtime() - rc0);   // wave clocks
        atomicAdd(&p.counters[27], (unsigned long long)rc_iters);          // attempt rounds (busiest lane)
        atomicAdd(&p.counters[28], 1ull);                                  // waves
        atomicAdd(&p.counters[8 + min(rc_iters, 15)], 1ull);               // waves by attempt rounds
        atomicMax(&p.counters[29], __builtin_amdgcn_s_memtime() - rc0);   // slowest wave
    }
#endif
    // this wave's consumption since the last refill: mgx_mt_slide_kernel, which follows every refill, sums
    // it over the waves into MtCtl.cons_last (the next launch's production ceiling)
    int csum = e < p.n ? cons : 0;
    for (int off = 32; off > 0; off >>= 1) csum += __shfl_xor(csum, off);
    if (tid == 0) {
        ulonglong4 b = p.blk[2 * p.nblk + blockIdx.x];   // (32-env waves: two slots per 64 envs)
        b.w = b.w > maxcur ? b.w : maxcur;
        b.x = (unsigned long long)csum;
        p.blk[2 * p.nblk + blockIdx.x] = b;
        if (err) atomicOr(p.err, err);
        if (p.clk.slots) clk_record(p.clk, CLK_REFILL, s_t0);   // (one wave per workgroup)
    }
}

template <int NW, bool EXT>
__global__ __launch_bounds__(64) void mgx_refill_kernel(KParams p) { refill_body<NW, EXT, false>(p); }
// The default variant (S <= 8, no EXT features) runs beside three step workgroups per CU:
// 176 + 3 x 112 VGPRs per SIMD lane fill the 512-entry file exactly.
template <>
__global__ __launch_bounds__(64, 3) void mgx_refill_kernel<1, false>(KParams p) {
    refill_body<1, false, false>(p);
}
// problem 'multi' without EXT features (every BASELINE config): the multi generator alone
template <int NW>
__global__ __launch_bounds__(64) void mgx_refill_multi_kernel(KParams p) { refill_body<NW, false, true>(p); }
template <>
__global__ __launch_bounds__(64, 3) void mgx_refill_multi_kernel<1>(KParams p) {
    refill_body<1, false, true>(p);
}
// ... at S = 8 (configs 2, 3 and 4): the grid size a constant -- room rectangles, the middle wall, the border
// masks and every cell index fold into immediates (round 4)
template <int EPW>
__global__ __launch_bounds__(64, 3) void mgx_refill_s8_kernel(KParams p) { refill_body<1, false, true, 8, EPW>(p); }

// ============================================================== scene kernel
// mgx_scene: regenerates env e's current episode from the RNG state its generation started from
// (inline mode keeps it, p.start_rng) and records what PlaygroundEnv's llm_description is built
// from (custom_env.py:122-2034): the objs list in placement order (doors, goal, keys flagged
// OBJ_KEYFLAG, objects), the agent, the mission and the generated grid (door lock bits).
// One lane; the generator is deterministic, so the record is exactly the episode in play.
template <int NW, bool EXT>
__global__ __launch_bounds__(64) void mgx_scene_kernel(KParams p, int64_t e, uint32_t *__restrict__ rec) {
    extern __shared__ __align__(16) uint8_t smem[];
    if (threadIdx.x != 0) return;
    uint8_t *s_grid = smem;
    uint8_t *s_scr = smem + ((64 * p.GSL + 15) & ~15);
    Gen<NW> G;
    load_gen(G, p, e, s_grid, s_scr, 0);
    const uint4 c0 = p.start_rng[2 * e], c1 = p.start_rng[2 * e + 1], inc = p.pcg[2 * e + 1];
    G.pcg.sh = ((uint64_t)c0.x << 32) | c0.y;
    G.pcg.sl = ((uint64_t)c0.z << 32) | c0.w;
    G.pcg.ih = ((uint64_t)inc.x << 32) | inc.y;
    G.pcg.il = ((uint64_t)inc.z << 32) | inc.w;
    G.pcg.uinteger = c1.x;
    G.pcg.has = c1.y & 1u;
    G.cur = (uint64_t)c1.z | ((uint64_t)c1.w << 32);
    G.gbase = ~0ull >> 1;
    ResetOut R;
    reset_env<NW, EXT>(G, R);
    rec[0] = (uint32_t)G.nobjs;
    rec[1] = (uint32_t)G.ax | ((uint32_t)G.ay << 8) | ((uint32_t)G.adir << 16);
    rec[2] = (uint32_t)R.mission_id | ((uint32_t)R.tx << 8) | ((uint32_t)R.ty << 16) | ((uint32_t)R.ta << 24);
    rec[3] = (uint32_t)R.livelocks;
    rec[4] = G.err;
    for (int k = 0; k < MAX_OBJS; k++) rec[8 + k] = k < G.nobjs ? G.objs[k] : 0u;
    for (int k = 0; k < p.S * p.S; k++) reinterpret_cast<uint8_t *>(rec + 8 + MAX_OBJS)[k] = G.g[k];
}

// ============================================================== MT ring slider
// One MT19937 block (624 words) generated in place by a workgroup: the sequential twist
// (CPython _random.c genrand_uint32) in three data-parallel phases, each read-all -> barrier ->
// write-all.  new[i] mixes s[i], s[i+1] and x[i] = s[i+397] (i < 227: the old word) or new[i-227]
// (i >= 227, written by the previous phase); i = 623 takes the new s[0].
__device__ __forceinline__ uint32_t mt_mix(uint32_t a, uint32_t b, uint32_t x) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return x ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}
__device__ __forceinline__ void mt_twist_block(uint32_t *s, int tid) {   // >= 227 threads
    uint32_t v = 0;
    if (tid < 227) v = mt_mix(s[tid], s[tid + 1], s[tid + 397]);
    __syncthreads();
    if (tid < 227) s[tid] = v;
    __syncthreads();
    const int i = 227 + tid;
    if (tid < 227) v = mt_mix(s[i], s[i + 1], s[i - 227]);
    __syncthreads();
    if (tid < 227) s[i] = v;
    __syncthreads();
    const int k = 454 + tid;
    if (tid < 170) v = mt_mix(s[k], s[k == 623 ? 0 : k + 1], s[k - 227]);
    __syncthreads();
    if (tid < 170) s[k] = v;
    __syncthreads();
}
__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    return y ^ (y >> 18);
}

// Extends the MT ring (MtCtl above).  Pass 1, every workgroup: the minimum live cursor of its
// SLIDE_ENVS envs -> atomicMin; the last workgroup to finish (fenced counter) runs pass 2: while the
// ring has room above that minimum, generate whole super-blocks (3,120 words = 312 groups) into the
// slots of groups no env can read again, at most MT_SLIDE_MAX_SB per launch.  Runs at every refill
// fork on the refill stream, right before mgx_refill_kernel (and before every inline generation,
// ring disabled): the launch sequence depends only on the call count (hipGraph-capturable); a
// launch with nothing to extend costs one 16-KB read pass per 4,096 envs.
__global__ __launch_bounds__(SLIDE_THREADS) void mgx_mt_slide_kernel(KParams p) {
    __shared__ uint32_t s_st[624];
    __shared__ uint8_t s_f[MT_SB_WORDS];
    __shared__ unsigned long long s_red[SLIDE_THREADS / 64], s_red2[SLIDE_THREADS / 64];
    __shared__ unsigned long long s_hi;
    __shared__ int s_nsb;
    const int tid = threadIdx.x;
    MtCtl *c = p.mtc;
    __shared__ unsigned long long s_t0;           // kernel clock: this workgroup's start
    if (p.clk.slots && tid == 0) s_t0 = clk_now();
    unsigned long long mn = ~0ull, mx = 0;
    const int64_t e0 = (int64_t)blockIdx.x * SLIDE_ENVS;
    // Every load of the thread's 16 envs first, then the stores: with a store between them (the ring_pubn copy)
    // each load group also waited for the store before it (vmcnt counts both on gfx9) -- 16 store round trips
    // per thread (round 4).
    constexpr int EPT = SLIDE_ENVS / SLIDE_THREADS;
    rpos_t tl[EPT];
    unsigned long long cu[EPT], pc[EPT];
#pragma unroll
    for (int k = 0; k < EPT; k++) {
        const int64_t e = e0 + k * SLIDE_THREADS + tid;
        const bool in = e < p.n;
        const int64_t ec = in ? e : 0;
        tl[k] = p.D > 0 ? p.ring_tail[ec] : (rpos_t)0;
        const uint2 cr = reinterpret_cast<const uint2 *>(p.cur_rng + 2 * ec + 1)[1];   // .z, .w: the MT cursor
        const uint2 ax = reinterpret_cast<const uint2 *>(p.aux + ec)[1];             // producer cursor
        cu[k] = in ? ((unsigned long long)cr.x | ((unsigned long long)cr.y << 32)) : ~0ull;
        pc[k] = in ? ((unsigned long long)ax.x | ((unsigned long long)ax.y << 32)) : 0ull;
    }
#pragma unroll
    for (int k = 0; k < EPT; k++) {
        const int64_t e = e0 + k * SLIDE_THREADS + tid;
        if (e < p.n) {
            if (p.D > 0) p.ring_pubn[e] = tl[k];           // the refill before this slide has completed
            unsigned long long v = cu[k];
            if (p.start_rng) {
                const uint4 sr = p.start_rng[2 * e + 1];
                const unsigned long long u = (unsigned long long)sr.z | ((unsigned long long)sr.w << 32);
                v = u < v ? u : v;
            }
            mn = v < mn ? v : mn;
            mx = pc[k] > mx ? pc[k] : mx;
        }
    }
    // prefix records of the stream positions generated by the slides before this one (round 6): this launch's
    // threads take PFX_PER_THREAD positions each from rec_done on, up to the last word a record may read
    unsigned long long rec_lo = 0, rec_hi = 0;
    if (p.pfx) {
        rec_lo = c->rec_done;
        const unsigned long long top = c->hi * (unsigned long long)MT_FIELDS;
        rec_hi = top > (unsigned long long)PFX_LOOK ? top - PFX_LOOK : 0ull;
        const unsigned long long T = (unsigned long long)gridDim.x * SLIDE_THREADS;
        for (int k = 0; k < PFX_PER_THREAD; k++) {
            const unsigned long long pos = rec_lo + (unsigned long long)blockIdx.x * SLIDE_THREADS + tid + k * T;
            if (pos < rec_hi) p.pfx[pfx_index(pos, p.mt_mask)] = pfx_compute(p, pos);
        }
    }
    // the refill waves' consumption (mgx_refill_kernel writes it in its workgroup stats): one per 64 envs
    unsigned long long cs = 0;
    if (tid < SLIDE_ENVS / 64) {
        const int64_t b = e0 / 64 + tid;
        if (b < p.nblk) {
            const int per = 64 / p.refill_epw;                // refill waves per 64 envs (1, 2 or 4)
            for (int k = 0; k < per; k++) cs += p.blk[2 * p.nblk + per * b + k].x;
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(mn, off), q = __shfl_xor(mx, off);
        mn = o < mn ? o : mn;
        mx = q > mx ? q : mx;
        cs += __shfl_xor(cs, off);
    }
    if ((tid & 63) == 0) { s_red[tid >> 6] = mn; s_red2[tid >> 6] = mx; }
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < SLIDE_THREADS / 64; w++) {
            mn = s_red[w] < mn ? s_red[w] : mn;
            mx = s_red2[w] > mx ? s_red2[w] : mx;
        }
        // The reductions are ordered before this workgroup's done-counter increment either by __threadfence()
        // (MGX_SLIDE_FENCE, the product: every workgroup and the last one write back their XCD's L2 -- buffer_wbl2)
        // or by waiting for the returning atomics (each has been performed at the device-scope coherence point when
        // its value is back; everything the last workgroup reads of this pass it reads with atomics, MtCtl's plain
        // fields come from earlier kernels).  Round 5 A/B: the fenced slide is the faster PIPELINE (the next refill
        // runs ~5-10 % faster after the write-back), although the fence-free slide itself is shorter.
        const unsigned long long r0 = atomicMin(&c->span_min, mn);
        const unsigned long long r1 = atomicMax(&c->span_max, mx);
        const unsigned long long r2 = cs ? atomicAdd(&c->cons_run, cs) : 0ull;   // (wave 0 holds this workgroup's blocks)
        if (MGX_SLIDE_FENCE) __threadfence();
        else asm volatile("" ::"v"(r0), "v"(r1), "v"(r2));                     // (waits for the three returns)
        s_nsb = atomicAdd(&c->done, 1u) == gridDim.x - 1 ? 1 : -1;   // last workgroup: pass 2
    }
    __syncthreads();
    if (s_nsb < 0) {
        if (p.clk.slots && tid == 0) clk_record(p.clk, CLK_SLIDE, s_t0);
        return;
    }
    if (tid == 0) {
        if (MGX_SLIDE_FENCE) __threadfence();
        const unsigned long long cons = atomicExch(&c->cons_run, 0ull);   // the last refill's consumption, all envs
        c->cons_last = cons;
        if (cons && p.D > 0 && p.n > 0) {
            // Round cap of the next refill (round 4): target production per env per epoch =
            // mean consumption + a margin m, so the lanes' levels drift up by m per epoch and only rarely
            // fall to the invariant's 2K (need-driven rounds).  A lane's deficit is a random walk with
            // per-epoch variance ~ mean (resets are ~Bernoulli per step); with drift m its stationary tail
            // is ~exp(-2 m x / mean), so m = 9 mean / (D - 2K) puts the 2K floor >= 18 e-folds away.  At
            // E = 64 (D = 256) that is 10.0 rounds (round 3's ceil(mean + 1/4) = 10 too); at the 20-step
            // epochs of the driver's line 3.04 (round 3: 4), i.e. 3 rounds in 24 epochs of 25.
            const double mean = (double)cons / (double)p.n;
            const double slack = (double)max(p.D - 2 * p.K, 1);
            const double tgt = mean * (1.0 + 9.0 / slack);
            const unsigned long long acc0 = c->round_acc;
            const unsigned long long acc1 = acc0 + (unsigned long long)(tgt * 1024.0 + 0.5);
            const int r = (int)((acc1 >> 10) - (acc0 >> 10));
            c->round_acc = acc1;
            c->round_cap = r > 1 ? r : 1;
        }
        if (p.pfx) {                                  // the positions every workgroup covered (rec_lo, hi as read by all)
            const unsigned long long T = (unsigned long long)gridDim.x * SLIDE_THREADS * PFX_PER_THREAD;
            c->rec_done = rec_lo + T < rec_hi ? rec_lo + T : (rec_hi > rec_lo ? rec_hi : rec_lo);
        }
        const unsigned long long m = atomicExch(&c->span_min, ~0ull);   // every workgroup's extremes; reset
        const unsigned long long x = atomicExch(&c->span_max, 0ull);
        c->done = 0;
        const unsigned long long cap = p.mt_mask + 1, hi = c->hi, need_lo = m / MT_FIELDS;
        const unsigned long long want_hi = (x + MT_AHEAD) / MT_FIELDS;    // generated this far ahead ...
        int nsb = 0;                                                      // ... within the ring above need_lo
        while (nsb < MT_SLIDE_MAX_SB && hi + (unsigned long long)nsb * MT_SB_GROUPS < want_hi &&
               hi + (unsigned long long)(nsb + 1) * MT_SB_GROUPS <= need_lo + cap)
            nsb++;
        s_hi = hi;
        s_nsb = nsb;
    }
    __syncthreads();
    const int nsb = s_nsb;
    if (nsb == 0) {
        if (p.clk.slots && tid == 0) clk_record(p.clk, CLK_SLIDE, s_t0);
        return;
    }
    for (int i = tid; i < 624; i += SLIDE_THREADS) s_st[i] = c->st[i];
    __syncthreads();
    unsigned long long hi = s_hi;
    for (int sb = 0; sb < nsb; sb++) {
        for (int b = 0; b < MT_SB_WORDS / 624; b++) {
            mt_twist_block(s_st, tid);
            for (int i = tid; i < 624; i += SLIDE_THREADS)
                s_f[b * 624 + i] = (uint8_t)(mt_temper(s_st[i]) >> 27);   // getrandbits(k<=5) field
        }
        __syncthreads();
        for (int gi = tid; gi < MT_SB_GROUPS; gi += SLIDE_THREADS) {
            uint64_t grp = 0;
#pragma unroll
            for (int k = 0; k < MT_FIELDS; k++) grp |= (uint64_t)s_f[gi * MT_FIELDS + k] << (6 * k);
            const uint64_t slot = (hi + (unsigned long long)gi) & p.mt_mask;
            p.mt[slot] = grp;
            if (slot < (uint64_t)MT_PAD) p.mt[p.mt_mask + 1 + slot] = grp;   // mirror: windows stay contiguous
        }
        __syncthreads();                                   // s_f is rewritten by the next super-block
        hi += MT_SB_GROUPS;
    }
    for (int i = tid; i < 624; i += SLIDE_THREADS) c->st[i] = s_st[i];
    if (tid == 0) {
        c->hi = hi;
        c->lo = hi > p.mt_mask + 1 ? hi - (p.mt_mask + 1) : 0;
        if (p.clk.slots) clk_record(p.clk, CLK_SLIDE, s_t0);
    }
}

// ================================================================ GAE kernel
// DictRolloutBuffer.compute_returns_and_advantage (SB3; fp32, numpy op order,
// built with -ffp-contract=off):  delta = ((r + (g*nv)*nnt) - V);  last = delta + (c*nnt)*last
// One workgroup of 256 threads per 64 columns (envs).  The recurrence is serial in t and must
// round exactly like the sequential numpy loop, so one wave (lane = column) computes it; the
// other three waves only load.  Tiles of GAE_TT steps, walked from t = T-1 down: while wave 0
// computes tile k from LDS (and stores adv/ret straight to HBM, coalesced), every thread already
// has its share of tile k+1 in flight in registers (float4 loads), written to LDS after the
// compute -- 64 x GAE_TT x 9 B per workgroup in flight, ~37 MB across the GPU at N = 65,536
// (a lane-per-column walk keeps at most 63 loads per wave in flight: latency-bound).
// DONES: the compact form -- `es` is u8 dones[T][N] (done after step t), next_non_terminal(t) =
// 1 - dones[t]; otherwise SB3's f32 episode_starts[T][N] plus last_dones (next_non_terminal(t)
// = 1 - episode_starts[t+1], 1 - last_dones at T-1).
constexpr int GAE_TT = 64;                 // steps per tile
typedef float gf4 __attribute__((ext_vector_type(4)));
constexpr int GAE_SHARDS = 256;
static_assert(GAE_SHARDS * 2 == MGX_GAE_SCRATCH_WORDS, "scratch size (include/mgx.h)");
__device__ double g_gae_shard[GAE_SHARDS][2];   // (sum A, sum A^2) partials when the caller passes no scratch

template <bool DONES>
__global__ __launch_bounds__(256, 4) void mgx_gae_kernel(const float *__restrict__ r, const float *__restrict__ v,
                                                      const void *__restrict__ es, const float *__restrict__ lv,
                                                      const uint8_t *__restrict__ ld, int64_t T, int64_t N, float g,
                                                      float c, float *__restrict__ adv, float *__restrict__ ret,
                                                      double *__restrict__ stats, double *__restrict__ shard) {
    __shared__ float s_r[GAE_TT][64], s_v[GAE_TT][64];
    __shared__ uint32_t s_e[GAE_TT][16];                 // flags as bytes (4 columns per dword)
    const int tid = threadIdx.x;
    const int64_t col0 = (int64_t)blockIdx.x * 64;
    const int ncol = (int)min<int64_t>(64, N - col0);
    // this thread's share of a tile: rows ri + 16 * m (m < 4), columns cj .. cj+3
    const int cj = (tid & 15) * 4, ri = tid >> 4;
    const bool vec = (N & 3) == 0 && cj + 4 <= ncol;      // 16-B aligned, whole quad in range
    gf4 pr[4], pv[4], pe[4];
    auto load_tile = [&](int64_t thi) {                   // rows t = thi - i, i < GAE_TT
#pragma unroll
        for (int m = 0; m < 4; m++) {
            const int64_t t = thi - (ri + 16 * m);
            pr[m] = pv[m] = pe[m] = gf4{0.f, 0.f, 0.f, 0.f};
            if (t < 0) continue;
            const int64_t k = t * N + col0 + cj;
            if (vec) {
                pr[m] = __builtin_nontemporal_load(reinterpret_cast<const gf4 *>(r + k));
                pv[m] = __builtin_nontemporal_load(reinterpret_cast<const gf4 *>(v + k));
                if (DONES) {
                    const uint32_t d = __builtin_nontemporal_load(reinterpret_cast<const uint32_t *>(
                        static_cast<const uint8_t *>(es) + k));
                    pe[m] = gf4{(float)(d & 0xFF), (float)((d >> 8) & 0xFF), (float)((d >> 16) & 0xFF),
                                (float)(d >> 24)};
                } else {
                    pe[m] = __builtin_nontemporal_load(reinterpret_cast<const gf4 *>(static_cast<const float *>(es) + k));
                }
            } else {
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    if (cj + q < ncol) {
                        pr[m][q] = r[k + q];
                        pv[m][q] = v[k + q];
                        pe[m][q] = DONES ? (float)static_cast<const uint8_t *>(es)[k + q]
                                         : static_cast<const float *>(es)[k + q];
                    }
                }
            }
        }
    };
    auto store_tile = [&]() {
#pragma unroll
        for (int m = 0; m < 4; m++) {
            const int i = ri + 16 * m;
            *reinterpret_cast<gf4 *>(&s_r[i][cj]) = pr[m];
            *reinterpret_cast<gf4 *>(&s_v[i][cj]) = pv[m];
            s_e[i][cj >> 2] = (uint32_t)pe[m][0] | ((uint32_t)pe[m][1] << 8) | ((uint32_t)pe[m][2] << 16) |
                              ((uint32_t)pe[m][3] << 24);
        }
    };
    // wave 0 state (lane = column)
    const int lane = tid & 63;
    const int64_t col = col0 + lane;
    const bool active = tid < 64 && lane < ncol;
    float last = 0.0f, nnt = 0.0f, nv = 0.0f;
    if (active) {
        nnt = DONES ? 0.0f : 1.0f - (float)ld[col];
        nv = lv[col];
    }
    double s1 = 0.0, s2 = 0.0;
    load_tile(T - 1);
    store_tile();
    __syncthreads();
    for (int64_t thi = T - 1; thi >= 0; thi -= GAE_TT) {
        const bool more = thi - GAE_TT >= 0;
        if (more) load_tile(thi - GAE_TT);                // next tile in flight during the compute
        if (active) {
            const int nrow = (int)min<int64_t>(GAE_TT, thi + 1);
#pragma unroll 8
            for (int i = 0; i < nrow; i++) {
                const int64_t k = (thi - i) * N + col;
                const float vt = s_v[i][lane], rt = s_r[i][lane];
                const float et = (float)reinterpret_cast<const uint8_t *>(&s_e[i][0])[lane];
                if (DONES) nnt = 1.0f - et;
                const float delta = (rt + (g * nv) * nnt) - vt;
                last = delta + (c * nnt) * last;
                __builtin_nontemporal_store(last, adv + k);
                __builtin_nontemporal_store(last + vt, ret + k);
                s1 += (double)last;
                s2 += (double)last * (double)last;
                if (!DONES) nnt = 1.0f - et;                // for step t-1: 1 - episode_starts[t]
                nv = vt;
            }
        }
        __syncthreads();                                  // wave 0 is done reading this tile
        if (more) {
            store_tile();
            __syncthreads();
        }
    }
    if (stats && tid < 64) {                              // wave 0 holds the sums
        for (int off = 32; off > 0; off >>= 1) {
            s1 += __shfl_down(s1, off);
            s2 += __shfl_down(s2, off);
        }
        if (tid == 0) {                                   // sharded: 1024 workgroups on 3 addresses would
            double *sh = shard + 2 * (blockIdx.x & (GAE_SHARDS - 1));   // serialise at L2 (~40 us)
            atomicAdd(&sh[0], s1);
            atomicAdd(&sh[1], s2);
        }
    }
}

// Folds the shards into stats (sum A, sum A^2, count += T*N) and re-zeroes them; runs right after
// mgx_gae_kernel on the same stream (GAE calls that accumulate stats are stream-ordered).
__global__ __launch_bounds__(GAE_SHARDS) void mgx_gae_reduce_kernel(double *__restrict__ stats, double *__restrict__ shard,
                                                                      double count) {
    __shared__ double red[2][GAE_SHARDS / 64];
    const int tid = threadIdx.x;
    double a = shard[2 * tid], b = shard[2 * tid + 1];
    shard[2 * tid] = 0.0;
    shard[2 * tid + 1] = 0.0;
    for (int off = 32; off > 0; off >>= 1) {
        a += __shfl_down(a, off);
        b += __shfl_down(b, off);
    }
    if ((tid & 63) == 0) { red[0][tid >> 6] = a; red[1][tid >> 6] = b; }
    __syncthreads();
    if (tid == 0) {
        for (int k = 1; k < GAE_SHARDS / 64; k++) { a += red[0][k]; b += red[1][k]; }
        atomicAdd(&stats[0], a);
        atomicAdd(&stats[1], b);
        atomicAdd(&stats[2], count);
    }
}

// ==================================================== synthetic random policy
// mgx_random_actions: out[i] = uniform on {0 .. n_actions - 1} from a counter-based hash of (seed, launch counter, i)
// -- splitmix64 twice, then Lemire's multiply-shift of the high 32 bits (bias < n / 2^32) -- so that a launch
// captured once in a hipGraph draws fresh actions at every replay: the counter lives in device memory and the last
// workgroup to finish advances it (every workgroup has read it by then: each reads it before its own tally add).
// Integer hashing, coalesced dword stores: 4 B written per action (HBM-bound, ~1 us per 10^6 actions).
__global__ __launch_bounds__(256) void mgx_random_actions_kernel(int32_t *__restrict__ out, int64_t count,
                                                                  uint32_t n_actions, uint64_t seed,
                                                                  unsigned long long *ctr) {
    const unsigned long long c = *reinterpret_cast<volatile unsigned long long *>(ctr);
    const uint64_t key = splitmix64(seed + (uint64_t)c * 0x9E3779B97F4A7C15ull);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += stride) {
        const uint64_t h = splitmix64(key ^ ((uint64_t)i * 0xD1B54A32D192ED03ull));
        out[i] = (int32_t)(((h >> 32) * (uint64_t)n_actions) >> 32);
    }
    __syncthreads();                                   // every thread of this workgroup has read the counter
    if (threadIdx.x == 0) {
        __threadfence();
        if (atomicAdd(reinterpret_cast<unsigned int *>(ctr + 1), 1u) == gridDim.x - 1) {
            *reinterpret_cast<volatile unsigned long long *>(ctr) = c + 1ull;   // (vector store)
            *reinterpret_cast<volatile unsigned int *>(ctr + 1) = 0u;
            __threadfence();
        }
    }
}

// ========================================================= compact layout kernels
// mgx_observe_compact: the current observation of every env as a compact row (byte 0
// direction, bytes 1..147 the [c][vx][vy] frame) + mission id -- e.g. right after mgx_reset,
// the first row of a compact rollout buffer.  One env per lane, from the engine state.
__global__ __launch_bounds__(256) void mgx_observe_kernel(KParams p, uint8_t *__restrict__ rows, uint8_t *__restrict__ mids) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= p.n) return;
    const EnvState st = p.state[e];
    uint8_t *row = rows + e * (int64_t)FROW;
    render_view(p.grid + e * p.GS, p.S, st.ax, st.ay, st.dir, st.carry, [&](int k, uint32_t v) {
        row[1 + k] = (uint8_t)v;
        row[1 + 49 + k] = (uint8_t)(v >> 8);
        row[1 + 98 + k] = (uint8_t)(v >> 16);
    });
    if (p.vis) apply_vis(row + 1);                 // this thread's own global writes: read back coherently
    row[0] = st.dir;
    mids[e] = st.mission_id;
}

// mgx_gather: SB3 stacked observations (VecTransposeImage + VecFrameStack(n_stack)) rebuilt
// from compact rows.  Sample b's newest frame is row index[b] (flat row*N + env) -- or, with
// `newest` (terminal rows [N][148]), env's terminal row, the older frames then starting at
// row index[b] itself.  Older slot k (1 <= k < n_stack) holds the row k steps back while no
// episode start lies in between (starts[row] = 1: that row is an episode's first
// observation), else zeros -- VecFrameStack's reset zeroing.  Outputs per sample: image
// [3*n_stack][7][7] (u8, or f32 = u8 / 255 as SB3 preprocess_obs), direction one-hot
// [4*n_stack] (u8 or f32), mission tokens [32*n_stack] (u8).  f32 = u8 * (1/255 in fp32): what
// torch's `x.float() / 255.0` computes on the GPU (division by a scalar as a reciprocal multiply).
// One workgroup per GATHER_TILE samples: phase A stages every needed row in LDS (dword loads,
// coalesced along a row; rows are 148 B = 37 dwords), phase B writes the tile's outputs,
// which are contiguous in memory, with consecutive threads on consecutive dwords.
constexpr int GATHER_TILE = 16;
constexpr int GATHER_MAXK = 8;
template <int K, bool F32>   // n_stack and output type are compile-time: every index split is a constant division
__global__ __launch_bounds__(256) void mgx_gather_kernel(const uint8_t *__restrict__ rows, const uint8_t *__restrict__ mids,
                                                         const uint8_t *__restrict__ starts, int64_t N, int64_t R,
                                                         const int64_t *__restrict__ index, int64_t B,
                                                         const uint8_t *__restrict__ newest,
                                                         const uint8_t *__restrict__ mtok, void *__restrict__ img_out,
                                                         void *__restrict__ dir_out, uint8_t *__restrict__ mis_out) {
    constexpr int img_f32 = F32, dir_f32 = F32;
    __shared__ uint32_t s_row[GATHER_TILE * K * (FROW / 4)];             // zeros where the slot is empty
    __shared__ int s_mid[GATHER_TILE * K];                               // -1: empty slot
    const int tid = threadIdx.x;
    const int64_t b0 = (int64_t)blockIdx.x * GATHER_TILE;
    const int nb = (int)min<int64_t>(GATHER_TILE, B - b0);
    const int npair = nb * K;
    // phase A1: per (sample, slot): source row and validity
    __shared__ const uint8_t *s_src[GATHER_TILE * K];
    if (tid < npair) {
        const int bi = tid / K, k = tid - bi * K;                        // k = slot (K-1 = newest)
        const int64_t idx = index[b0 + bi];
        const int64_t row0 = idx / N, env = idx - row0 * N;
        // flat index of the row j steps before the newest: linear buffer (R = 0), or a ring of R rows
        // (mgx_gather_ring: the rows wrap, so a rollout's history rows need no copy)
        const auto back_idx = [&](int j) -> int64_t {
            int64_t r = row0 - j;
            if (R > 0 && r < 0) r += ((-r + R - 1) / R) * R;
            return r * N + env;
        };
        const int back = K - 1 - k;                                      // steps back from the newest
        const uint8_t *src = nullptr;
        int mid = -1;
        if (newest) {
            // newest = terminal row; older slot j back = row idx - (j-1)*N, valid while no start
            // among rows idx .. idx - (j-2)*N (the terminal row itself continues the episode)
            if (back == 0) { src = newest + env * FROW; mid = mids[idx]; }
            else {
                bool ok = true;
                for (int j = 0; j < back - 1 && ok; j++) ok = !starts[back_idx(j)];
                if (ok) { const int64_t r = back_idx(back - 1); src = rows + r * FROW; mid = mids[r]; }
            }
        } else {
            bool ok = true;
            for (int j = 0; j < back && ok; j++) ok = !starts[back_idx(j)];
            if (ok) { const int64_t r = back_idx(back); src = rows + r * FROW; mid = mids[r]; }
        }
        s_src[tid] = src;
        s_mid[tid] = mid;
    }
    __syncthreads();
    // phase A2: stage the rows (37 dwords each)
    constexpr int RW = FROW / 4;
    for (int i = tid; i < npair * RW; i += blockDim.x) {
        const int pr = i / RW, w = i - pr * RW;
        const uint8_t *src = s_src[pr];
        s_row[pr * RW + w] = src ? reinterpret_cast<const uint32_t *>(src)[w] : 0u;
    }
    __syncthreads();
    const uint8_t *s_b = reinterpret_cast<const uint8_t *>(s_row);
    // phase B1: images -- sample bi, output byte o = slot o / 147, frame byte o % 147 (row byte 1 + ...)
    constexpr int IMGB = FRAME * K;
    const int nbytes = nb * IMGB;
    if (img_f32) {
        float4 *out = reinterpret_cast<float4 *>(static_cast<float *>(img_out) + b0 * IMGB);
        for (int q = tid; q < (nbytes >> 2); q += blockDim.x) {
            float v[4];
#pragma unroll
            for (int t = 0; t < 4; t++) {
                const int o = 4 * q + t, bi = o / IMGB, ob = o - bi * IMGB, k = ob / FRAME, f = ob - k * FRAME;
                v[t] = (float)s_b[(bi * K + k) * FROW + 1 + f] * (1.0f / 255.0f);
            }
            out[q] = make_float4(v[0], v[1], v[2], v[3]);
        }
        for (int o = (nbytes & ~3) + tid; o < nbytes; o += blockDim.x) {
            const int bi = o / IMGB, ob = o - bi * IMGB, k = ob / FRAME, f = ob - k * FRAME;
            static_cast<float *>(img_out)[b0 * IMGB + o] = (float)s_b[(bi * K + k) * FROW + 1 + f] * (1.0f / 255.0f);
        }
    } else {
        uint8_t *out = static_cast<uint8_t *>(img_out) + b0 * IMGB;
        // the tile's output is 4-B aligned when IMGB is (n_stack multiple of 4: whole dwords)
        const bool al = ((b0 * IMGB) & 3) == 0;
        for (int q = tid; q < (nbytes >> 2); q += blockDim.x) {
            uint32_t w = 0;
#pragma unroll
            for (int t = 0; t < 4; t++) {
                const int o = 4 * q + t, bi = o / IMGB, ob = o - bi * IMGB, k = ob / FRAME, f = ob - k * FRAME;
                w |= (uint32_t)s_b[(bi * K + k) * FROW + 1 + f] << (8 * t);
            }
            if (al) reinterpret_cast<uint32_t *>(out)[q] = w;
            else for (int t = 0; t < 4; t++) out[4 * q + t] = (uint8_t)(w >> (8 * t));
        }
        for (int o = (nbytes & ~3) + tid; o < nbytes; o += blockDim.x) {
            const int bi = o / IMGB, ob = o - bi * IMGB, k = ob / FRAME, f = ob - k * FRAME;
            out[o] = s_b[(bi * K + k) * FROW + 1 + f];
        }
    }
    // phase B2: direction one-hot (slot k: 4 values) and mission tokens (slot k: 32 tokens)
    for (int i = tid; i < npair * 4; i += blockDim.x) {
        const int pr = i >> 2, c = i & 3;
        const bool on = s_mid[pr] >= 0 && s_b[pr * FROW] == c;
        const int64_t o = (b0 + pr / K) * (int64_t)(4 * K) + (pr % K) * 4 + c;
        if (dir_f32) static_cast<float *>(dir_out)[o] = on ? 1.0f : 0.0f;
        else static_cast<uint8_t *>(dir_out)[o] = on ? 1 : 0;
    }
    for (int i = tid; i < npair * 8; i += blockDim.x) {
        const int pr = i >> 3, c = i & 7;                                // 8 dwords of 4 tokens
        const int mid = s_mid[pr];
        const uint32_t v = mid >= 0 ? reinterpret_cast<const uint32_t *>(mtok + mid * 32)[c] : 0u;
        reinterpret_cast<uint32_t *>(mis_out + (b0 + pr / K) * (int64_t)(32 * K) + (pr % K) * 32)[c] = v;
    }
}

// ================================================================== host side
thread_local std::string g_last_error;

mgx_status fail(mgx_status s, const std::string &msg) {
    g_last_error = msg;
    return s;
}
#define HIP_TRY(expr)                                                                                  \
    do {                                                                                               \
        hipError_t _e = (expr);                                                                        \
        if (_e != hipSuccess) return fail(MGX_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

// CPython random.seed(n) -> MT19937 init_by_array(32-bit chunks of n)
struct HostMT {
    uint32_t mt[624];
    int mti;
    void init_genrand(uint32_t s) {
        mt[0] = s;
        for (int i = 1; i < 624; i++) mt[i] = 1812433253U * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
        mti = 624;
    }
    void seed(uint64_t n) {
        uint32_t key[2];
        int klen = 0;
        if (n == 0) key[klen++] = 0;
        while (n) { key[klen++] = (uint32_t)n; n >>= 32; }
        init_genrand(19650218U);
        int i = 1, j = 0, k = 624 > klen ? 624 : klen;
        for (; k; k--) {
            mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525U)) + key[j] + (uint32_t)j;
            i++; j++;
            if (i >= 624) { mt[0] = mt[623]; i = 1; }
            if (j >= klen) j = 0;
        }
        for (k = 623; k; k--) {
            mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941U)) - (uint32_t)i;
            i++;
            if (i >= 624) { mt[0] = mt[623]; i = 1; }
        }
        mt[0] = 0x80000000U;
    }
    uint32_t next() {
        static const uint32_t mag01[2] = {0U, 0x9908b0dfU};
        uint32_t y;
        if (mti >= 624) {
            int kk;
            for (kk = 0; kk < 624 - 397; kk++) {
                y = (mt[kk] & 0x80000000U) | (mt[kk + 1] & 0x7fffffffU);
                mt[kk] = mt[kk + 397] ^ (y >> 1) ^ mag01[y & 1U];
            }
            for (; kk < 623; kk++) {
                y = (mt[kk] & 0x80000000U) | (mt[kk + 1] & 0x7fffffffU);
                mt[kk] = mt[kk + (397 - 624)] ^ (y >> 1) ^ mag01[y & 1U];
            }
            y = (mt[623] & 0x80000000U) | (mt[0] & 0x7fffffffU);
            mt[623] = mt[396] ^ (y >> 1) ^ mag01[y & 1U];
            mti = 0;
        }
        y = mt[mti++];
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680U;
        y ^= (y << 15) & 0xefc60000U;
        y ^= (y >> 18);
        return y;
    }
};

// TokenizeVocabWrapper vocab (environment.py:75-81): ' ' '\n' '-' ':' ',' '.' a..z
void tokenize(const std::string &s, uint8_t out[32]) {
    std::memset(out, 0, 32);
    for (size_t i = 0; i < s.size() && i < 32; i++) {
        char c = s[i];
        if (c >= 'A' && c <= 'Z') c = (char)(c - 'A' + 'a');
        int v = 0;
        switch (c) {
            case ' ': v = 0; break; case '\n': v = 1; break; case '-': v = 2; break;
            case ':': v = 3; break; case ',': v = 4; break; case '.': v = 5; break;
            default: v = (c >= 'a' && c <= 'z') ? 6 + (c - 'a') : 0;
        }
        out[i] = (uint8_t)v;
    }
}

const char *CMD_TXT[3] = {"go to", "toggle", "pick up"};
const char *CN_TXT[6] = {"blue", "green", "grey", "purple", "red", "yellow"};
const char *TS_TXT[4] = {"door", "key", "ball", "box"};

const char *DIR_TXT[4] = {"left", "right", "up", "down"};

bool mission_text(int id, std::string &out) {
    if (id < 0 || id > 255) return false;
    if (id == MID_DROP) { out = "drop"; return true; }
    if (id >= MID_MOVE && id < MID_MOVE + 4) { out = std::string("move ") + DIR_TXT[id - MID_MOVE]; return true; }
    if (id >= 128) return false;
    int cmd = id & 3, cn = (id >> 2) & 7, ts = (id >> 5) & 3;
    if (cmd == CMD_GOTOGOAL) { out = "go to goal"; return id == CMD_GOTOGOAL; }
    if (cn > 5) return false;
    out = std::string(CMD_TXT[cmd]) + " " + CN_TXT[cn] + " " + TS_TXT[ts];
    return true;
}

}  // namespace

struct mgx_handle {
    mgx_config cfg;
    int device;
    KParams kp;
    size_t lds_step, lds_step_compact, lds_reset, lds_refill, lds_rollout, lds_rollout32;
    int roll_epb;           // envs per fused-rollout block: 64, or 32 at S = 16 (MGX_ROLL_EPB_S16)
    int nw;                 // 64-bit words of the generator's S*S cell masks (1, 2 or 4)
    bool ext;               // generator variant with full / drp / mov / obstacles
    int refill_every;       // K: steps per refill epoch
    uint64_t calls;         // mgx_step calls since the last mgx_reset
    uint64_t resets;        // mgx_reset calls since create
    uint64_t refill_launches;  // refill kernels enqueued since create (incl. the synchronous initial fills)
    bool seed_pending;      // mgx_set_seed called since the last reset
    bool in_flight;         // a refill (and the slide after it) forked and not yet joined
    bool pub_stale;         // ring_pub not yet copied from ring_tail this epoch (mgx_step_kernel reads it)
    bool serial_refill;     // diagnostics (env MGX_SERIAL_REFILL=1): refill on the caller's stream
    bool refill_multi;      // problem 'multi' without EXT features refills with mgx_refill_multi_kernel
                            // (round 2: the all-problems kernel measured the same speed)
    hipStream_t side;       // refill stream
    hipEvent_t ev_fork, ev_done;
    void *allocs[19];       // [17]: mgx_set_random_policy's per-workgroup launch counters, [18] prefix records
    uint32_t *scene_dev;    // mgx_scene's record (inside allocs[15], inline mode only)
};

extern "C" {

const char *mgx_last_error(void) { return g_last_error.c_str(); }
int mgx_abi_version(void) { return MGX_ABI_VERSION; }

mgx_status mgx_mission_text(int mission_id, char *buf, size_t buflen) {
    std::string s;
    if (!mission_text(mission_id, s)) return fail(MGX_ERR_INVALID, "invalid mission id");
    if (!buf || buflen < s.size() + 1) return fail(MGX_ERR_INVALID, "buffer too small");
    std::memcpy(buf, s.c_str(), s.size() + 1);
    return MGX_OK;
}

// range(floor((size - 2)**2 * percent_obstacles)) (custom_env.py:156), fp64 like Python
static int n_obstacles_of(const mgx_config *c) {
    if (!c->obstacles) return 0;
    return (int)std::floor((double)((c->size - 2) * (c->size - 2)) * c->percent_obstacles);
}

static mgx_status validate(const mgx_config *c) {
    if (!c) return fail(MGX_ERR_INVALID, "null config");
    if (c->size < 5 || c->size > 16) return fail(MGX_ERR_INVALID, "size must be in 5..16");
    if (c->n_envs <= 0) return fail(MGX_ERR_INVALID, "n_envs must be > 0");
    if (c->n_stack < 1 || c->n_stack > 8) return fail(MGX_ERR_INVALID, "n_stack must be in 1..8");
    if (c->obstacles && !(c->percent_obstacles >= 0.0 && c->percent_obstacles <= 1.0))
        return fail(MGX_ERR_INVALID, "percent_obstacles must be in [0, 1]");
    const int interior = (c->size - 2) * (c->size - 2);
    const int nobst = n_obstacles_of(c);
    switch (c->problem) {
        case MGX_PROBLEM_MULTI:
            if (!(c->mission == -1 || c->mission == 0 || c->mission == 1 || c->mission == 2 || c->mission == 5))
                return fail(MGX_ERR_INVALID, "multi: mission must be None, 0, 1, 2 or 5");
            if (c->num_objects > 18) return fail(MGX_ERR_INVALID, "Number of objects to be generated is more than the available objects.");
            break;
        case MGX_PROBLEM_GTO: case MGX_PROBLEM_GTG:
            if (c->num_objects > 24) return fail(MGX_ERR_INVALID, "Number of objects to be generated is more than the available objects.");
            break;
        case MGX_PROBLEM_OPN:
            if (c->num_objects > 12) return fail(MGX_ERR_INVALID, "Number of objects to be generated is more than the available objects.");
            break;
        case MGX_PROBLEM_PKP:
            if (c->num_objects > 18) return fail(MGX_ERR_INVALID, "Number of objects to be generated is more than the available objects.");
            break;
        case MGX_PROBLEM_DRP: case MGX_PROBLEM_MOV:
            if (c->num_objects > 24) return fail(MGX_ERR_INVALID, "Number of objects to be generated is more than the available objects.");
            break;
        case MGX_PROBLEM_FULL:
            break;
        default:
            return fail(MGX_ERR_INVALID, "Invalid problem type given");
    }
    if (c->num_objects < 0) return fail(MGX_ERR_INVALID, "num_objects must be >= 0");
    if (c->problem != MGX_PROBLEM_MULTI) {
        // single room: every object, [goal], the agent and each obstacle take one free interior
        // cell via place_obj, which never gives up (max_tries=inf): more than fit = a hang
        const bool goal = c->problem == MGX_PROBLEM_GTG || c->problem == MGX_PROBLEM_DRP || c->problem == MGX_PROBLEM_FULL;
        const int cells = (c->problem == MGX_PROBLEM_FULL ? 24 : c->num_objects) + (goal ? 1 : 0) + 1 + nobst;
        if (cells > interior)
            return fail(MGX_ERR_INVALID, "the room cannot hold the objects, goal, agent and obstacles "
                                         "(the reference's place_obj would never return)");
    }
    if (c->terminal_mode < 0 || c->terminal_mode > 2) return fail(MGX_ERR_INVALID, "bad terminal_mode");
    return MGX_OK;
}

mgx_status mgx_create(const mgx_config *cfg, int device, mgx_handle **out) {
    if (!out) return fail(MGX_ERR_INVALID, "null out");
    *out = nullptr;
    mgx_status s = validate(cfg);
    if (s != MGX_OK) return s;
    int prev = 0;
    HIP_TRY(hipGetDevice(&prev));
    HIP_TRY(hipSetDevice(device));
    mgx_handle *h = new (std::nothrow) mgx_handle();
    if (!h) return fail(MGX_ERR_OOM, "host alloc");
    h->cfg = *cfg;
    h->device = device;
    if (h->cfg.livelock_words <= 0) h->cfg.livelock_words = MGX_LIVELOCK_WORDS;
    // default depth 512 (round 6; 256 since round 3, 128 before).  A lane's ring level is a random walk
    // (consumption i.i.d. per epoch, variance ~ its mean) reflected at D, with the drift the production ceiling
    // gives it (mgx_mt_slide_kernel: mean x (1 + 9 / (D - 2K)), 18 e-folds of the walk's tail between D and
    // the invariant's floor 2K).  At D = 256 and the driver's 20-step epochs that target is 3.04 episodes per
    // epoch: one epoch in ~28 ran a fourth attempt round (the launch +33 %).  At D = 512 it is 2.97 -- three
    // rounds every epoch, with 22 e-folds of the tail at the integer rounding's own drift.  4.3 GB of rings at
    // 65,536 envs (S = 8), 21 GB at config 5's 131,072 x 16 x 16 (288 GB of HBM)
    if (h->cfg.ring_depth == 0) h->cfg.ring_depth = 512;
    if (h->cfg.ring_depth < 0) {
        h->cfg.ring_depth = 0;                                   // ring disabled: every reset generated inline
    } else {
        int d = 2;
        while (d < h->cfg.ring_depth && d < MGX_MAX_RING) d <<= 1;   // power of two (mod-2^16 ring indices)
        h->cfg.ring_depth = d;
    }
    if (h->cfg.refill_every <= 0) h->cfg.refill_every = std::max(1, std::min(h->cfg.ring_depth / 4, 64));
    if (h->cfg.refill_every > h->cfg.ring_depth / 2) h->cfg.refill_every = std::max(1, h->cfg.ring_depth / 2);
    // default production cap: ~1.3x a random policy's consumption (1 in 7 steps ends an episode on
    // 'done' alone; 0.146 resets per env-step measured at config 2), i.e. 6 at the default epoch of 32
    if (h->cfg.refill_cap == 0) h->cfg.refill_cap = std::max(2, (h->cfg.refill_every * 19 + 50) / 100);
    h->refill_every = h->cfg.refill_every;
    h->calls = 0;
    h->in_flight = false;
    h->pub_stale = true;
    // scheduling choices: compile-time (mgx_diag.h; A/B builds), never read from the environment
    h->serial_refill = MGX_SERIAL_REFILL != 0;
    // refill waves at issue priority 2 over co-resident step / rollout waves: the refill sets the
    // pipeline beside the fused rollout (+3-7 % at config 2, +4 % at config 4; per-step layouts
    // and config 5 within +-0.5 %, round 3)
    h->kp.refill_prio = MGX_REFILL_PRIO;
    h->refill_multi = true;
    // MT ring: a power of two of 10-word groups holding at least mt_table_words words (>= 512 groups)
    if (h->cfg.mt_table_words <= 0) h->cfg.mt_table_words = (int64_t)1 << 26;
    int64_t ring_groups = 512;
    while (ring_groups * MT_FIELDS < h->cfg.mt_table_words && ring_groups < ((int64_t)1 << 26)) ring_groups <<= 1;
    h->cfg.mt_table_words = ring_groups * MT_FIELDS;
    const int64_t N = cfg->n_envs;
    const int S = cfg->size;
    const int GS = ((S * S) + 15) & ~15;
    const int IMG = FRAME * cfg->n_stack;
    // initial fill: whole super-blocks, MT_HOST_FILL words at most (the slider generates the rest)
    const int64_t hi0 = std::min(ring_groups * MT_FIELDS, (int64_t)MT_HOST_FILL) / MT_SB_WORDS * MT_SB_GROUPS;

    auto bail = [&](mgx_status st) {
        for (void *&p : h->allocs) if (p) { (void)hipFree(p); p = nullptr; }
        delete h;
        (void)hipSetDevice(prev);
        return st;
    };
    size_t sizes[6] = {(size_t)N * sizeof(EnvState), (size_t)N * GS, (size_t)N * 32, (size_t)N * 16,
                       (size_t)(ring_groups + MT_PAD) * 8, 256 * 32 + 64};
    for (int i = 0; i < 6; i++) {
        hipError_t e = hipMalloc(&h->allocs[i], sizes[i]);
        if (e != hipSuccess) return bail(fail(MGX_ERR_OOM, std::string("hipMalloc: ") + hipGetErrorString(e)));
    }
    const int D = h->cfg.ring_depth;
    {
        const size_t REC = (size_t)((GS + 48 + 63) & ~63);
        size_t rs[5] = {(size_t)N * D * REC, 16, 16, (size_t)N * 32, (size_t)N * 5 * sizeof(rpos_t) + 64};
        for (int i = 0; i < 5; i++) {
            hipError_t e = hipMalloc(&h->allocs[7 + i], rs[i] ? rs[i] : 16);
            if (e != hipSuccess) return bail(fail(MGX_ERR_OOM, std::string("hipMalloc ring: ") + hipGetErrorString(e)));
        }
        hipError_t e = hipMemset(h->allocs[11], 0, (size_t)N * 5 * sizeof(rpos_t) + 64);
        if (e != hipSuccess) return bail(fail(MGX_ERR_HIP, "hipMemset ring ctl"));
        e = hipMemset(h->allocs[10], 0, (size_t)N * 32);      // cursors read by the MT slider before any reset
        if (e == hipSuccess) e = hipMemset(h->allocs[3], 0, (size_t)N * 16);
        if (e != hipSuccess) return bail(fail(MGX_ERR_HIP, "hipMemset RNG state"));
        e = hipMalloc(&h->allocs[12], (size_t)N * 4 + 64);
        if (e != hipSuccess) return bail(fail(MGX_ERR_OOM, "hipMalloc fix list"));
        e = hipMemset(h->allocs[12], 0, (size_t)N * 4 + 64);
        if (e != hipSuccess) return bail(fail(MGX_ERR_HIP, "hipMemset fix list"));
    }
    {
        hipError_t e = hipMalloc(&h->allocs[6], MGX_NCOUNTERS * sizeof(unsigned long long) + 64);
        if (e != hipSuccess) return bail(fail(MGX_ERR_OOM, "hipMalloc counters"));
        e = hipMemset(h->allocs[6], 0, MGX_NCOUNTERS * sizeof(unsigned long long) + 64);
        if (e != hipSuccess) return bail(fail(MGX_ERR_HIP, "hipMemset counters"));
    }
    // MT19937(base_seed) output stream as packed top-5-bit fields (mgx_device.h: randbelow): the
    // ring's first hi0 groups + the mirror pad, and the generator state after them (MtCtl), from
    // which mgx_mt_slide_kernel continues the stream on the device
    {
        std::vector<uint64_t> tab((size_t)hi0, 0ull);            // slots [hi0, ring) are written before read
        HostMT m;
        m.seed((uint64_t)cfg->base_seed);
        for (int64_t i = 0; i < hi0 * MT_FIELDS; i++) {
            const uint64_t f = m.next() >> 27;
            tab[(size_t)(i / MT_FIELDS)] |= f << (6 * (i % MT_FIELDS));
        }
        hipError_t e = hipMemcpy(h->allocs[4], tab.data(), tab.size() * 8, hipMemcpyHostToDevice);
        if (e == hipSuccess)                                       // mirror pad = slots 0 .. MT_PAD-1
            e = hipMemcpy((uint64_t *)h->allocs[4] + ring_groups, tab.data(), (size_t)MT_PAD * 8, hipMemcpyHostToDevice);
        if (e != hipSuccess) return bail(fail(MGX_ERR_HIP, "upload MT table"));
        MtCtl c;
        std::memset(&c, 0, sizeof c);
        c.lo = 0;
        c.hi = (unsigned long long)hi0;
        c.span_min = ~0ull;
        c.span_max = 0;
        std::memcpy(c.st, m.mt, sizeof c.st);         // hi0 * 10 words = whole blocks: m.mti == 624
        e = hipMalloc(&h->allocs[16], sizeof(MtCtl));
        if (e != hipSuccess) return bail(fail(MGX_ERR_OOM, "hipMalloc MT ring control"));
        e = hipMemcpy(h->allocs[16], &c, sizeof c, hipMemcpyHostToDevice);
        if (e != hipSuccess) return bail(fail(MGX_ERR_HIP, "upload MT ring control"));
    }
    {
        std::vector<uint8_t> tok(256 * 32 + 64, 0);
        for (int id = 0; id < 256; id++) {
            std::string s;
            if (mission_text(id, s)) tokenize(s, &tok[(size_t)id * 32]);
        }
        hipError_t e = hipMemcpy(h->allocs[5], tok.data(), tok.size(), hipMemcpyHostToDevice);
        if (e != hipSuccess) return bail(fail(MGX_ERR_HIP, "upload mission table"));
    }
    KParams &p = h->kp;
    p.state = (EnvState *)h->allocs[0];
    p.grid = (uint8_t *)h->allocs[1];
    p.pcg = (uint4 *)h->allocs[2];
    p.aux = (uint4 *)h->allocs[3];
    p.mt = (uint64_t *)h->allocs[4];
    p.mt_mask = (uint64_t)(ring_groups - 1);
    p.mtc = (MtCtl *)h->allocs[16];
    p.mtok = (const uint8_t *)h->allocs[5];
    p.counters = (unsigned long long *)h->allocs[6];
    p.err = (uint32_t *)((char *)h->allocs[6] + MGX_NCOUNTERS * sizeof(unsigned long long));
    p.n = N;
    p.seed_base = cfg->base_seed + cfg->env_index_offset;
    p.S = S;
    p.GS = GS;
    p.GSL = GS + 4;
    p.n_stack = cfg->n_stack;
    p.img_bytes = IMG;
    // objs list capacity: multi = doors (<= 4) + goal + keys (<= 4) + objects (the lower-left
    // room of the 3/4-room layouts reuses the upper-left counter, Q1: <= 2 x num_objects);
    // single room = objects (24 for 'full') + goal.  Sized per config: the refill's LDS
    // per wave decides how many step workgroups fit beside it on a CU.
    p.obj_cap = std::min(MAX_OBJS, cfg->problem == MGX_PROBLEM_MULTI ? 9 + 2 * cfg->num_objects
                                   : (cfg->problem == MGX_PROBLEM_FULL ? 24 : cfg->num_objects) + 1);
    // (>= 12 words: the refill stages each episode's header + RNG snapshot in the lane's objs list once the
    // attempt is done, for the wave's coalesced record write)
    p.obj_stride = std::max(p.obj_cap, 12) | 1;
    const int nw_ = S * S <= 64 ? 1 : (S * S <= 128 ? 2 : 4);   // generator variant (h->nw below)
    const int scratch = BLOCK_ENVS * scratch_per_env(p.obj_stride, nw_);
    p.stk_lds = (std::max(BLOCK_ENVS * IMG, scratch) + 15) & ~15;   // reset kernel: stack area doubles as scratch
    p.grid_lds = (BLOCK_ENVS * (GS + 4) + 15) & ~15;
    p.fast_roll = cfg->n_stack == 4;
    // (the compact layout always uses [64][148] frame rows, also at n_stack 1)
    p.stk_step = (std::max(BLOCK_ENVS * FROW, p.fast_roll ? 0 : BLOCK_ENVS * IMG) + 15) & ~15;
    p.problem = cfg->problem;
    p.cfg_mission = cfg->mission;
    p.num_objects = cfg->num_objects;
    p.all_doors_open = cfg->all_doors_open;
    p.llw = (uint32_t)h->cfg.livelock_words;
    p.terminal_mode = cfg->terminal_mode;
    p.n_obstacles = n_obstacles_of(cfg);
    p.vis = cfg->see_through_walls ? 0 : 1;
    p.has_move = (cfg->problem == MGX_PROBLEM_MOV || cfg->problem == MGX_PROBLEM_FULL) ? 1 : 0;
    p.manual = cfg->manual ? 1 : 0;
    p.ring_rec = (uint8_t *)h->allocs[7];
    p.REC = (GS + 48 + 63) & ~63;
    p.cur_rng = (uint4 *)h->allocs[10];
    p.ring_head = (rpos_t *)h->allocs[11];
    p.ring_tail = p.ring_head + N;
    p.ring_pub = p.ring_head + 2 * N;
    p.ring_seen = p.ring_head + 3 * N;
    p.ring_pubn = p.ring_head + 4 * N;
    p.fix_list = (uint32_t *)h->allocs[12];
    p.fix_count = p.fix_list + N + 4;       // 16-B aligned tail of the same allocation
    p.fix_done = p.fix_list + N + 8;
    p.nblk = (int)((N + 63) / 64);
    {
        // 32-env refill waves when 64-env ones would not give every SIMD one (config 4: 512 waves for
        // 1,024 SIMDs); MGX_REFILL_EPW forces 32 or 64
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 256;
        p.refill_epw = MGX_REFILL_EPW == 16 || MGX_REFILL_EPW == 32 || MGX_REFILL_EPW == 64 ? MGX_REFILL_EPW
                                                                                       : (p.nblk < 4 * cus ? 32 : 64);
    }
    {
        // sections: [0, nblk) steps, [nblk, 2 nblk) fixup, [2 nblk, 6 nblk) refill waves (64 / refill_epw
        // per 64 envs)
        hipError_t e = hipMalloc(&h->allocs[13], (size_t)6 * p.nblk * sizeof(ulonglong4));
        if (e != hipSuccess) return bail(fail(MGX_ERR_OOM, "hipMalloc stats"));
        e = hipMemset(h->allocs[13], 0, (size_t)6 * p.nblk * sizeof(ulonglong4));
        if (e != hipSuccess) return bail(fail(MGX_ERR_HIP, "hipMemset stats"));
        p.blk = (ulonglong4 *)h->allocs[13];
    }
    {   // 'move' target_range words: current episode [N] + ring [N][D] (16 B when unused)
        const bool mv = cfg->problem == MGX_PROBLEM_MOV || cfg->problem == MGX_PROBLEM_FULL;
        const size_t bytes = mv ? (size_t)N * (1 + (size_t)D) * 8 : 16;
        hipError_t e = hipMalloc(&h->allocs[14], bytes);
        if (e != hipSuccess) return bail(fail(MGX_ERR_OOM, "hipMalloc move ranges"));
        e = hipMemset(h->allocs[14], 0, bytes);
        if (e != hipSuccess) return bail(fail(MGX_ERR_HIP, "hipMemset move ranges"));
        p.range_cur = (uint64_t *)h->allocs[14];
        p.ring_range = mv ? p.range_cur + N : p.range_cur;
    }
    p.D = D;
    p.start_rng = nullptr;
    p.rnd_ctr = nullptr;                   // random policy off (mgx_set_random_policy)
    p.rnd_seed = 0;
    p.pfx = nullptr;                       // prefix records: multi-room problems with the ring (below)
    p.mt_shift = 0;
    while ((1ll << p.mt_shift) < ring_groups) p.mt_shift++;
    if (D == 0) {   // inline mode: keep each episode's generation start state (mgx_scene) + its record
        const size_t bytes = (size_t)N * 32 + MGX_SCENE_WORDS * sizeof(uint32_t);
        hipError_t e = hipMalloc(&h->allocs[15], bytes);
        if (e != hipSuccess) return bail(fail(MGX_ERR_OOM, "hipMalloc start rng"));
        e = hipMemset(h->allocs[15], 0, bytes);
        if (e != hipSuccess) return bail(fail(MGX_ERR_HIP, "hipMemset start rng"));
        p.start_rng = (uint4 *)h->allocs[15];
        h->scene_dev = (uint32_t *)((char *)h->allocs[15] + (size_t)N * 32);
    }
    p.K = h->cfg.refill_every;
    p.cap = h->cfg.refill_cap;
    p.initial_fill = 0;
    p.mission64 = cfg->mission_int64;
    h->lds_step = (size_t)p.stk_step + (size_t)BLOCK_ENVS * 2 * GS   // grids + popped grids (chunk-major)
                  + (size_t)BLOCK_ENVS * 5 * 16;                      // + popped header, 2 token halves, RNG snapshot
    h->lds_reset = (size_t)p.stk_lds + (size_t)p.grid_lds;
    HIP_TRY(hipFuncSetAttribute((const void *)mgx_step_kernel<int32_t, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_step));
    HIP_TRY(hipFuncSetAttribute((const void *)mgx_step_kernel<int64_t, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_step));
    HIP_TRY(hipFuncSetAttribute((const void *)mgx_step_kernel<int32_t, false, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_step));
    HIP_TRY(hipFuncSetAttribute((const void *)mgx_step_kernel<int64_t, false, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_step));
    h->lds_step_compact = (size_t)((BLOCK_ENVS * FROW + 15) & ~15) + (size_t)BLOCK_ENVS * 2 * GS   // frame rows + grids
                          + (size_t)BLOCK_ENVS * 3 * 16;                                     // + popped header, RNG snapshot
    HIP_TRY(hipFuncSetAttribute((const void *)mgx_step_kernel<int32_t, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_step_compact));
    HIP_TRY(hipFuncSetAttribute((const void *)mgx_step_kernel<int64_t, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_step_compact));
    HIP_TRY(hipFuncSetAttribute((const void *)mgx_step_kernel<int32_t, true, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_step_compact));
    HIP_TRY(hipFuncSetAttribute((const void *)mgx_step_kernel<int64_t, true, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_step_compact));
    // fused rollout: frame rows + current grids + two staged ring episodes (grid, header) + actions
    // [+ 'move' target ranges]
    const auto roll_lds = [&](int epb) {
        return (size_t)((epb * FROW + 15) & ~15) + (size_t)epb * 3 * GS + (size_t)epb * 2 * 16 + (size_t)2 * epb * 4 +
               ((cfg->problem == MGX_PROBLEM_MOV || cfg->problem == MGX_PROBLEM_FULL) ? (size_t)epb * 8 : 0) +
               (size_t)MGX_ROLL_LDS_PAD;
    };
    h->lds_rollout = roll_lds(64);
    h->lds_rollout32 = roll_lds(32);
    h->roll_epb = (S == 16 && MGX_ROLL_EPB_S16 == 32) ? 32 : 64;
#define MGX_ROLL_LDS(V, M, R)                                                                                     \
    HIP_TRY(hipFuncSetAttribute((const void *)mgx_rollout_kernel<V, M, R>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                (int)h->lds_rollout))
    MGX_ROLL_LDS(false, false, false); MGX_ROLL_LDS(false, false, true); MGX_ROLL_LDS(false, true, false);
    MGX_ROLL_LDS(false, true, true); MGX_ROLL_LDS(true, false, false); MGX_ROLL_LDS(true, false, true);
    MGX_ROLL_LDS(true, true, false); MGX_ROLL_LDS(true, true, true);
    HIP_TRY(hipFuncSetAttribute((const void *)mgx_rollout_kernel<false, false, false, 8>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_rollout));
    HIP_TRY(hipFuncSetAttribute((const void *)mgx_rollout_kernel<false, false, true, 8>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_rollout));
    HIP_TRY(hipFuncSetAttribute((const void *)mgx_rollout_kernel<false, false, false, 16, 32>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_rollout32));
    HIP_TRY(hipFuncSetAttribute((const void *)mgx_rollout_kernel<false, false, true, 16, 32>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_rollout32));
#undef MGX_ROLL_LDS
    h->nw = S * S <= 64 ? 1 : (S * S <= 128 ? 2 : 4);
    h->ext = cfg->obstacles || cfg->problem == MGX_PROBLEM_FULL || cfg->problem == MGX_PROBLEM_DRP ||
             cfg->problem == MGX_PROBLEM_MOV;
    // fewer envs per refill wave only where the S = 8 refill kernel runs (launch_refill); every other refill
    // kernel is 64 envs per wave, and the slide reads its stats by that count
    if (!(h->refill_multi && !h->ext && p.problem == MGX_PROBLEM_MULTI && h->nw == 1 && S == 8))
        p.refill_epw = 64;
#define MGX_SET_LDS1(K, bytes) \
    HIP_TRY(hipFuncSetAttribute((const void *)K, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(bytes)))
#define MGX_SET_LDS(K, bytes)                                                                  \
    MGX_SET_LDS1((K<1, false>), bytes); MGX_SET_LDS1((K<2, false>), bytes); MGX_SET_LDS1((K<4, false>), bytes); \
    MGX_SET_LDS1((K<1, true>), bytes); MGX_SET_LDS1((K<2, true>), bytes); MGX_SET_LDS1((K<4, true>), bytes)
    MGX_SET_LDS(mgx_reset_kernel, h->lds_reset);
    h->lds_refill = (size_t)((64 * (GS + 4) + 15) & ~15) + (size_t)64 * scratch_per_env(p.obj_stride, h->nw);
    MGX_SET_LDS(mgx_refill_kernel, h->lds_refill);
    MGX_SET_LDS1(mgx_refill_multi_kernel<1>, h->lds_refill); MGX_SET_LDS1(mgx_refill_multi_kernel<2>, h->lds_refill);
    MGX_SET_LDS1(mgx_refill_multi_kernel<4>, h->lds_refill);
    MGX_SET_LDS1(mgx_refill_s8_kernel<64>, h->lds_refill);
    MGX_SET_LDS1(mgx_refill_s8_kernel<32>, h->lds_refill);
    MGX_SET_LDS1(mgx_refill_s8_kernel<16>, h->lds_refill);
    MGX_SET_LDS(mgx_fixup_kernel, h->lds_refill);
    MGX_SET_LDS(mgx_scene_kernel, h->lds_refill);
#undef MGX_SET_LDS
#undef MGX_SET_LDS1
    {
        hipError_t e = hipStreamCreateWithFlags(&h->side, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&h->ev_done, hipEventDisableTiming);
        if (e != hipSuccess) return bail(fail(MGX_ERR_HIP, "side stream / events"));
    }
    if (MGX_PFX_MEMO && cfg->problem == MGX_PROBLEM_MULTI && D > 0) {
        // prefix records (round 6): one u64 per word of the MT ring (671 MB at the default 2^26-word ring), zeroed (no
        // record), then the records of the host-generated start of the stream; the slides keep them a pass behind
        const size_t words = (size_t)ring_groups * MT_FIELDS;
        hipError_t e = hipMalloc(&h->allocs[18], words * sizeof(uint64_t));
        if (e != hipSuccess) return bail(fail(MGX_ERR_OOM, "hipMalloc prefix records"));
        e = hipMemset(h->allocs[18], 0, words * sizeof(uint64_t));
        if (e != hipSuccess) return bail(fail(MGX_ERR_HIP, "hipMemset prefix records"));
        p.pfx = (uint64_t *)h->allocs[18];
        const long long top = hi0 * MT_FIELDS - PFX_LOOK;
        if (top > 0) {
            hipLaunchKernelGGL(mgx_prefix_kernel, dim3(1024), dim3(256), 0, 0, p, 0ull, (unsigned long long)top);
            e = hipGetLastError();
            if (e == hipSuccess) {
                const unsigned long long rd = (unsigned long long)top;
                e = hipMemcpy((char *)h->allocs[16] + offsetof(MtCtl, rec_done), &rd, sizeof rd, hipMemcpyHostToDevice);
            }
            if (e == hipSuccess) e = hipDeviceSynchronize();
            if (e != hipSuccess) return bail(fail(MGX_ERR_HIP, "prefix records"));
        }
    }
    (void)hipSetDevice(prev);
    *out = h;
    return MGX_OK;
}

mgx_status mgx_destroy(mgx_handle *h) {
    if (!h) return MGX_OK;
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(h->device);
    if (h->side) {
        (void)hipStreamSynchronize(h->side);
        (void)hipStreamDestroy(h->side);
    }
    if (h->ev_fork) (void)hipEventDestroy(h->ev_fork);
    if (h->ev_done) (void)hipEventDestroy(h->ev_done);
    for (void *&p : h->allocs) if (p) { (void)hipFree(p); p = nullptr; }
    (void)hipSetDevice(prev);
    delete h;
    return MGX_OK;
}

// Launch generator kernel K<NW, EXT> for this handle's mask width and feature variant.
#define MGX_GEN_LAUNCH(K, ...)                                                                    \
    do {                                                                                          \
        const int v_ = h->nw | (h->ext ? 8 : 0);                                                  \
        if (v_ == 1) hipLaunchKernelGGL((K<1, false>), __VA_ARGS__);                              \
        else if (v_ == 2) hipLaunchKernelGGL((K<2, false>), __VA_ARGS__);                         \
        else if (v_ == 4) hipLaunchKernelGGL((K<4, false>), __VA_ARGS__);                         \
        else if (v_ == 9) hipLaunchKernelGGL((K<1, true>), __VA_ARGS__);                          \
        else if (v_ == 10) hipLaunchKernelGGL((K<2, true>), __VA_ARGS__);                         \
        else hipLaunchKernelGGL((K<4, true>), __VA_ARGS__);                                       \
    } while (0)

// Extends the MT ring ahead of the generator kernels that follow on `stream` (MtCtl).
static mgx_status launch_slide(mgx_handle *h, void *stream) {
    const unsigned g = (unsigned)((h->kp.n + SLIDE_ENVS - 1) / SLIDE_ENVS);
    hipLaunchKernelGGL(mgx_mt_slide_kernel, dim3(g), dim3(SLIDE_THREADS), 0, (hipStream_t)stream, h->kp);
    HIP_TRY(hipGetLastError());
    return MGX_OK;
}

// One refill launch, then the MT slide for the NEXT one (round 3: the slide used to precede its refill
// and held it back ~27 us per epoch beside a rollout).  `done`: event recorded after both.
static mgx_status launch_refill(mgx_handle *h, void *stream, hipEvent_t done = nullptr) {
    if (h->kp.D == 0) return MGX_OK;
    h->refill_launches++;
    const int64_t nblk = (h->kp.n + 63) / 64;
    if (h->refill_multi && !h->ext && h->kp.problem == MGX_PROBLEM_MULTI) {
        const dim3 g((unsigned)nblk), b(64);
        if (h->nw == 1 && h->kp.S == 8) {
            if (h->kp.refill_epw == 32)
                hipLaunchKernelGGL(mgx_refill_s8_kernel<32>, dim3((unsigned)((h->kp.n + 31) / 32)), b, h->lds_refill,
                                   (hipStream_t)stream, h->kp);
            else if (h->kp.refill_epw == 16)
                hipLaunchKernelGGL(mgx_refill_s8_kernel<16>, dim3((unsigned)((h->kp.n + 15) / 16)), b, h->lds_refill,
                                   (hipStream_t)stream, h->kp);
            else
                hipLaunchKernelGGL(mgx_refill_s8_kernel<64>, g, b, h->lds_refill, (hipStream_t)stream, h->kp);
        }
        else if (h->nw == 1) hipLaunchKernelGGL((mgx_refill_multi_kernel<1>), g, b, h->lds_refill, (hipStream_t)stream, h->kp);
        else if (h->nw == 2) hipLaunchKernelGGL((mgx_refill_multi_kernel<2>), g, b, h->lds_refill, (hipStream_t)stream, h->kp);
        else hipLaunchKernelGGL((mgx_refill_multi_kernel<4>), g, b, h->lds_refill, (hipStream_t)stream, h->kp);
    } else {
        MGX_GEN_LAUNCH(mgx_refill_kernel, dim3((unsigned)nblk), dim3(64), h->lds_refill, (hipStream_t)stream, h->kp);
    }
    HIP_TRY(hipGetLastError());
    // the next refill's window of the MT stream: generated ahead of the cursors this one left; the
    // slide also publishes this refill's tails (ring_pubn), so the epoch join (`done`) waits for it
    mgx_status ss = launch_slide(h, stream);
    if (ss != MGX_OK) return ss;
    if (done) HIP_TRY(hipEventRecord(done, (hipStream_t)stream));
    return MGX_OK;
}

// full: also the MT slide that follows the refill (mgx_join, mgx_reset: nothing of the handle's left
// running on the side stream); the epoch fork waits for the refill alone.
static mgx_status join_refill(mgx_handle *h, void *stream) {
    if (h->in_flight) {
        HIP_TRY(hipStreamWaitEvent((hipStream_t)stream, h->ev_done, 0));
        h->in_flight = false;
    }
    return MGX_OK;
}

// Epoch start: join the last refill (and the slide after it, which published its tails in ring_pubn),
// then fork this epoch's refill onto the side stream.  It writes only slots the steps cannot pop before
// the next publish, and RNG state only the refill uses.
// In two halves so that a caller can enqueue its own launch between them: fork_begin joins the previous
// epoch's refill and records the fork point on `stream`; fork_end launches this epoch's refill on the side
// stream from that point.  Whatever is launched on `stream` in between runs beside the refill, not after it.
static mgx_status fork_begin(mgx_handle *h, void *stream) {
    // the previous epoch's refill is joined here, not at that epoch's last step: work the caller
    // enqueues between epochs (GAE, the policy forward) runs beside the refill's tail.  No copy on this
    // stream: the fused rollout reads ring_pubn, the per-step calls copy it to ring_pub at their first
    // call (publish_for_steps)
    mgx_status js = join_refill(h, stream);
    if (js != MGX_OK) return js;
    h->pub_stale = true;
    if (h->serial_refill) return launch_refill(h, stream);
    HIP_TRY(hipEventRecord(h->ev_fork, (hipStream_t)stream));
    return MGX_OK;
}
static mgx_status fork_end(mgx_handle *h) {
    if (h->serial_refill) return MGX_OK;
    HIP_TRY(hipStreamWaitEvent(h->side, h->ev_fork, 0));
    mgx_status s = launch_refill(h, h->side, h->ev_done);
    if (s != MGX_OK) return s;
    h->in_flight = true;
    return MGX_OK;
}
static mgx_status fork_refill(mgx_handle *h, void *stream) {
    mgx_status s = fork_begin(h, stream);
    return s != MGX_OK ? s : fork_end(h);
}

// mgx_step_kernel pops below ring_pub, which must not move within a launch (its waves read it
// independently): a copy of ring_pubn made at the epoch's first per-step call (any byte it holds is a
// completed refill's tail).
static mgx_status publish_for_steps(mgx_handle *h, void *stream) {
    if (!h->pub_stale) return MGX_OK;
    HIP_TRY(hipMemcpyAsync(h->kp.ring_pub, h->kp.ring_pubn, (size_t)h->kp.n * sizeof(rpos_t), hipMemcpyDeviceToDevice,
                           (hipStream_t)stream));
    h->pub_stale = false;
    return MGX_OK;
}

static KOut make_out(const mgx_obs *obs, const mgx_step_out *so) {
    KOut o;
    std::memset(&o, 0, sizeof o);
    const mgx_obs *ob = so ? &so->obs : obs;
    o.img = (uint8_t *)ob->image_dev;
    o.dir = (uint8_t *)ob->direction_dev;
    o.mis = ob->mission_dev;
    if (so) {
        o.t_img = (uint8_t *)so->terminal.image_dev;
        o.t_dir = (uint8_t *)so->terminal.direction_dev;
        o.t_mis = so->terminal.mission_dev;
        o.reward = so->reward_dev;
        o.reward64 = so->reward64_dev;
        o.term = so->terminated_dev;
        o.trunc = so->truncated_dev;
        o.done = so->done_dev;
        o.ep_ret = so->ep_return_dev;
        o.ep_len = so->ep_len_dev;
        o.livelock = so->livelock_dev;
    }
    return o;
}

mgx_status mgx_reset(mgx_handle *h, const mgx_obs *obs, int32_t *livelock_dev, void *stream) {
    if (!h || !obs || !obs->image_dev || !obs->direction_dev || !obs->mission_dev)
        return fail(MGX_ERR_INVALID, "mgx_reset: null argument");
    KOut o = make_out(obs, nullptr);
    o.livelock = livelock_dev;
    {
        mgx_status js = join_refill(h, stream);  // a refill still running would race the reset
        if (js != MGX_OK) return js;
    }
    const int64_t nblk = (h->kp.n + BLOCK_ENVS - 1) / BLOCK_ENVS;
    h->kp.reset_mode = h->resets == 0 ? 0 : (h->seed_pending ? 1 : 2);
    h->resets++;
    h->seed_pending = false;
    MGX_GEN_LAUNCH(mgx_reset_kernel, dim3((unsigned)nblk), dim3(BLOCK_THREADS), h->lds_reset, (hipStream_t)stream, h->kp, o);
    HIP_TRY(hipGetLastError());
    h->calls = 0;
    h->kp.initial_fill = 1;                     // fills every ring to D (synchronously on `stream`)
    const mgx_status rs = launch_refill(h, stream);
    h->kp.initial_fill = 0;
    return rs;
}

mgx_status mgx_debug_counters(mgx_handle *h, void *stream, uint64_t *out, int n) {
    if (!h || !out || n < 0 || n > MGX_NCOUNTERS) return fail(MGX_ERR_INVALID, "bad argument");
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    HIP_TRY(hipStreamSynchronize(h->side));
    HIP_TRY(hipMemcpy(out, h->kp.counters, (size_t)n * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return MGX_OK;
}

mgx_status mgx_set_seed(mgx_handle *h, int64_t seed) {
    if (!h) return fail(MGX_ERR_INVALID, "null handle");
    h->kp.seed_base = seed + h->cfg.env_index_offset;
    h->seed_pending = true;
    return MGX_OK;
}

// grid of every launch of a clocked kernel class (the clock's per-workgroup records need one grid per class)
static int clock_groups(const mgx_handle *h, int cls) {
    const int64_t nblk = (h->kp.n + BLOCK_ENVS - 1) / BLOCK_ENVS;
    if (cls == CLK_STEP) return (int)nblk;
    if (cls == CLK_ROLL32) return h->roll_epb == 32 && h->kp.S == 16 ? (int)((h->kp.n + 31) / 32) : 0;
    if (cls == CLK_SLIDE) return (int)((h->kp.n + SLIDE_ENVS - 1) / SLIDE_ENVS);
    return (int)((h->kp.n + h->kp.refill_epw - 1) / h->kp.refill_epw);   // (64 except the S = 8 kernel's 32/16)
}

int64_t mgx_clock_words(const mgx_handle *h, int slots) {
    if (!h || slots < 1) return -1;
    int64_t w = 0;
    for (int c = 0; c < CLK_CLASSES; c++) w += (int64_t)clock_groups(h, c) * (1 + 2 * (int64_t)slots);
    return w;
}

int mgx_clock_groups(const mgx_handle *h, int cls) {
    if (!h || cls < 0 || cls >= CLK_CLASSES) return -1;
    return clock_groups(h, cls);
}

mgx_status mgx_set_clock(mgx_handle *h, uint64_t *clock_dev, int slots, int *tick_khz) {
    if (!h || (clock_dev && slots < 1)) return fail(MGX_ERR_INVALID, "mgx_set_clock: bad argument");
    static_assert(CLK_CLASSES == MGX_CLOCK_CLASSES, "include/mgx.h clock layout");
    KClock &k = h->kp.clk;
    std::memset(&k, 0, sizeof k);
    if (clock_dev) {
        unsigned long long *b = reinterpret_cast<unsigned long long *>(clock_dev);
        for (int c = 0; c < CLK_CLASSES; c++) {
            k.base[c] = b;
            k.groups[c] = clock_groups(h, c);
            b += (size_t)k.groups[c] * (1 + 2 * (size_t)slots);
        }
        k.slots = slots;
    }
    if (tick_khz) {
        int khz = 0;
        HIP_TRY(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, h->device));
        *tick_khz = khz;
    }
    return MGX_OK;
}

mgx_status mgx_get_config(const mgx_handle *h, mgx_config *out) {
    if (!h || !out) return fail(MGX_ERR_INVALID, "null argument");
    *out = h->cfg;
    return MGX_OK;
}

mgx_status mgx_join(mgx_handle *h, void *stream) {
    if (!h) return fail(MGX_ERR_INVALID, "null handle");
    return join_refill(h, stream);
}

mgx_status mgx_step(mgx_handle *h, const void *actions_dev, int action_bytes, const mgx_step_out *out, void *stream) {
    if (!h || !out || !actions_dev) return fail(MGX_ERR_INVALID, "mgx_step: null argument");
    if (!out->obs.image_dev || !out->obs.direction_dev || !out->obs.mission_dev || !out->reward_dev ||
        !out->terminated_dev || !out->truncated_dev)
        return fail(MGX_ERR_INVALID, "mgx_step: missing output buffer");
    if (h->kp.terminal_mode != MGX_TERMINAL_NONE &&
        (!out->terminal.image_dev || !out->terminal.direction_dev || !out->terminal.mission_dev))
        return fail(MGX_ERR_INVALID, "mgx_step: terminal_mode needs terminal buffers");
    if (action_bytes != 4 && action_bytes != 8) return fail(MGX_ERR_INVALID, "action_bytes must be 4 or 8");
    KOut o = make_out(nullptr, out);
    const int64_t nblk = (h->kp.n + BLOCK_ENVS - 1) / BLOCK_ENVS;
    if (h->kp.D > 0 && h->calls % (uint64_t)h->refill_every == 0) {
        mgx_status fs = fork_refill(h, stream);
        if (fs != MGX_OK) return fs;
    }
    if (h->kp.D > 0) {
        mgx_status ps = publish_for_steps(h, stream);
        if (ps != MGX_OK) return ps;
    }
    // S = 8 (configs 2, 3 and 4): the kernel compiled for the grid size (round 4)
#define MGX_STEP(A, C, SCV, LDS)                                                                                   \
    hipLaunchKernelGGL((mgx_step_kernel<A, C, SCV>), dim3((unsigned)nblk), dim3(BLOCK_THREADS), LDS, (hipStream_t)stream, \
                       h->kp, o, (const A *)actions_dev)
    const bool s8 = h->kp.S == 8;
    if (action_bytes == 4) {
        if (s8) MGX_STEP(int32_t, false, 8, h->lds_step); else MGX_STEP(int32_t, false, 0, h->lds_step);
    } else if (action_bytes == 8) {
        if (s8) MGX_STEP(int64_t, false, 8, h->lds_step); else MGX_STEP(int64_t, false, 0, h->lds_step);
    }
    HIP_TRY(hipGetLastError());
    if (h->kp.D == 0) {   // no ring: every done env is generated inline, right after the step
        mgx_status ss = launch_slide(h, stream);
        if (ss != MGX_OK) return ss;
        const unsigned fblk = (unsigned)h->kp.nblk;
        MGX_GEN_LAUNCH(mgx_fixup_kernel, dim3(fblk), dim3(64), h->lds_refill, (hipStream_t)stream, h->kp, o);
        HIP_TRY(hipGetLastError());
    }
    h->calls++;
    return MGX_OK;
}

mgx_status mgx_step_compact(mgx_handle *h, const void *actions_dev, int action_bytes, const mgx_compact_out *out,
                            void *stream) {
    if (!h || !out || !actions_dev) return fail(MGX_ERR_INVALID, "mgx_step_compact: null argument");
    if (!out->row_dev || !out->mission_id_dev || !out->reward_dev || !out->terminated_dev || !out->truncated_dev)
        return fail(MGX_ERR_INVALID, "mgx_step_compact: missing output buffer");
    if (h->kp.terminal_mode != MGX_TERMINAL_NONE && !out->terminal_row_dev)
        return fail(MGX_ERR_INVALID, "mgx_step_compact: terminal_mode needs terminal_row_dev");
    if (h->kp.D == 0) return fail(MGX_ERR_INVALID, "mgx_step_compact: needs the episode ring (ring_depth >= 0)");
    if (action_bytes != 4 && action_bytes != 8) return fail(MGX_ERR_INVALID, "action_bytes must be 4 or 8");
    KOut o;
    std::memset(&o, 0, sizeof o);
    o.img = out->row_dev;
    o.mis = out->mission_id_dev;
    o.t_img = out->terminal_row_dev;
    o.reward = out->reward_dev;
    o.reward64 = out->reward64_dev;
    o.term = out->terminated_dev;
    o.trunc = out->truncated_dev;
    o.done = out->done_dev;
    o.ep_ret = out->ep_return_dev;
    o.ep_len = out->ep_len_dev;
    o.livelock = out->livelock_dev;
    const int64_t nblk = (h->kp.n + BLOCK_ENVS - 1) / BLOCK_ENVS;
    if (h->calls % (uint64_t)h->refill_every == 0) {
        mgx_status fs = fork_refill(h, stream);
        if (fs != MGX_OK) return fs;
    }
    mgx_status ps = publish_for_steps(h, stream);
    if (ps != MGX_OK) return ps;
    const bool s8 = h->kp.S == 8;
    if (action_bytes == 4) {
        if (s8) MGX_STEP(int32_t, true, 8, h->lds_step_compact); else MGX_STEP(int32_t, true, 0, h->lds_step_compact);
    } else {
        if (s8) MGX_STEP(int64_t, true, 8, h->lds_step_compact); else MGX_STEP(int64_t, true, 0, h->lds_step_compact);
    }
#undef MGX_STEP
    HIP_TRY(hipGetLastError());
    h->calls++;
    return MGX_OK;
}

static double *gae_scratch(double *stats_scratch_dev);
static mgx_status rollout_impl(mgx_handle *h, const int32_t *actions_dev, int K, const mgx_rollout_out *out,
                               const mgx_gae_args *gae, void *stream) {
    if (!h || !out) return fail(MGX_ERR_INVALID, "mgx_rollout_compact: null argument");
    if (!actions_dev && !h->kp.rnd_ctr)
        return fail(MGX_ERR_INVALID, "mgx_rollout_compact: null actions_dev (and no mgx_set_random_policy)");
    if (!out->rows_dev || !out->mission_ids_dev || !out->rewards_dev || !out->terminated_dev || !out->truncated_dev ||
        !out->dones_dev)
        return fail(MGX_ERR_INVALID, "mgx_rollout_compact: missing output buffer");
    if (h->kp.terminal_mode != MGX_TERMINAL_NONE && !out->terminal_row_dev)
        return fail(MGX_ERR_INVALID, "mgx_rollout_compact: terminal_mode needs terminal_row_dev");
    if (h->kp.D == 0) return fail(MGX_ERR_INVALID, "mgx_rollout_compact: needs the episode ring (ring_depth >= 0)");
    const uint64_t E = (uint64_t)h->refill_every;
    if (K < 1 || (h->calls % E) + (uint64_t)K > E)
        return fail(MGX_ERR_INVALID, "mgx_rollout_compact: the K steps must lie within one refill epoch "
                                     "((calls % refill_every) + K <= refill_every)");
    ROut o;
    o.rows = out->rows_dev;
    o.mids = out->mission_ids_dev;
    o.t_rows = out->terminal_row_dev;
    o.reward = out->rewards_dev;
    o.reward64 = out->rewards64_dev;
    o.term = out->terminated_dev;
    o.trunc = out->truncated_dev;
    o.done = out->dones_dev;
    o.ep_ret = out->ep_return_dev;
    o.ep_len = out->ep_len_dev;
    o.livelock = out->livelock_dev;
    o.gv = o.glv = nullptr;
    o.gg = o.gc = 0.0f;
    o.gadv = o.gret = nullptr;
    o.gshard = nullptr;
    if (gae) {
        if (!gae->values_dev || !gae->last_values_dev || !gae->advantages_dev || !gae->returns_dev)
            return fail(MGX_ERR_INVALID, "mgx_rollout_compact_gae: missing GAE buffer");
        o.gv = gae->values_dev;
        o.glv = gae->last_values_dev;
        o.gg = gae->gamma;
        o.gc = gae->gamma_lambda;
        o.gadv = gae->advantages_dev;
        o.gret = gae->returns_dev;
        o.gshard = gae->adv_stats_dev ? gae_scratch(gae->stats_scratch_dev) : nullptr;
    }
    // Launch order of the epoch's refill and this rollout (both start from the same fork point):
    // refill first (round 4 A/B: with the rollout first, its workgroups took the CU
    // slots and the refill's waves, the longer of the two, started late (20-step line 4.0-4.2 vs
    // 5.2-5.4 x 10^9 env-steps/s, tools/gpu_r4_refill_ab.sh), although the rollout alone is shorter then).
    const bool fork = h->calls % E == 0;
    if (fork) {
        mgx_status fs = fork_refill(h, stream);
        if (fs != MGX_OK) return fs;
    }
    const int64_t nblk = (h->kp.n + BLOCK_ENVS - 1) / BLOCK_ENVS;
    const int var = (h->kp.vis ? 4 : 0) | (h->kp.has_move ? 2 : 0) | (o.reward64 ? 1 : 0);
#define MGX_ROLL(V, M, R, ...)                                                                                    \
    hipLaunchKernelGGL((mgx_rollout_kernel<V, M, R, ##__VA_ARGS__>), dim3((unsigned)nblk), dim3(ROLL_THREADS),   \
                       h->lds_rollout, (hipStream_t)stream, h->kp, o, actions_dev, K)
    // S = 16 (config 5) with 32-env blocks: grid and LDS of their own
#define MGX_ROLL32(R)                                                                                              \
    hipLaunchKernelGGL((mgx_rollout_kernel<false, false, R, 16, 32>), dim3((unsigned)((h->kp.n + 31) / 32)),         \
                       dim3(4 * 32 + 64), h->lds_rollout32, (hipStream_t)stream, h->kp, o, actions_dev, K)
    const bool r32 = h->roll_epb == 32 && h->kp.S == 16;
    switch (var) {
        // S = 8 (configs 2, 3 and 4): the grid size a constant (render and grid-copy address math in immediates)
        case 0:
            if (h->kp.S == 8) MGX_ROLL(false, false, false, 8);
            else if (r32) MGX_ROLL32(false);
            else MGX_ROLL(false, false, false, 0);
            break;
        case 1:
            if (h->kp.S == 8) MGX_ROLL(false, false, true, 8);
            else if (r32) MGX_ROLL32(true);
            else MGX_ROLL(false, false, true, 0);
            break;
        case 2: MGX_ROLL(false, true, false); break;
        case 3: MGX_ROLL(false, true, true); break;
        case 4: MGX_ROLL(true, false, false); break;
        case 5: MGX_ROLL(true, false, true); break;
        case 6: MGX_ROLL(true, true, false); break;
        default: MGX_ROLL(true, true, true); break;
    }
#undef MGX_ROLL
#undef MGX_ROLL32
    HIP_TRY(hipGetLastError());
    h->calls += (uint64_t)K;
    if (o.gshard) {   // fold the launch's GAE partials into the caller's triple (as mgx_gae_dones)
        hipLaunchKernelGGL(mgx_gae_reduce_kernel, dim3(1), dim3(GAE_SHARDS), 0, (hipStream_t)stream,
                           gae->adv_stats_dev, o.gshard, (double)K * (double)h->kp.n);
        HIP_TRY(hipGetLastError());
    }
    return MGX_OK;
}

mgx_status mgx_rollout_compact(mgx_handle *h, const int32_t *actions_dev, int K, const mgx_rollout_out *out,
                               void *stream) {
    return rollout_impl(h, actions_dev, K, out, nullptr, stream);
}

mgx_status mgx_rollout_compact_gae(mgx_handle *h, const int32_t *actions_dev, int K, const mgx_rollout_out *out,
                                   const mgx_gae_args *gae, void *stream) {
    if (!gae) return fail(MGX_ERR_INVALID, "mgx_rollout_compact_gae: null GAE arguments");
    return rollout_impl(h, actions_dev, K, out, gae, stream);
}

mgx_status mgx_observe_compact(mgx_handle *h, uint8_t *row_dev, uint8_t *mission_id_dev, void *stream) {
    if (!h || !row_dev || !mission_id_dev) return fail(MGX_ERR_INVALID, "mgx_observe_compact: null argument");
    const int64_t nblk = (h->kp.n + 255) / 256;
    hipLaunchKernelGGL(mgx_observe_kernel, dim3((unsigned)nblk), dim3(256), 0, (hipStream_t)stream, h->kp, row_dev,
                       mission_id_dev);
    HIP_TRY(hipGetLastError());
    return MGX_OK;
}

mgx_status mgx_gather(const mgx_handle *h, const uint8_t *rows_dev, const uint8_t *mission_ids_dev,
                      const uint8_t *starts_dev, int64_t n_envs, const int64_t *index_dev, int64_t n_samples,
                      const uint8_t *terminal_rows_dev, void *image_dev, int image_f32, void *direction_dev,
                      int direction_f32, uint8_t *mission_dev, void *stream) {
    return mgx_gather_ring(h, rows_dev, mission_ids_dev, starts_dev, n_envs, 0, index_dev, n_samples,
                           terminal_rows_dev, image_dev, image_f32, direction_dev, direction_f32, mission_dev, stream);
}

mgx_status mgx_gather_ring(const mgx_handle *h, const uint8_t *rows_dev, const uint8_t *mission_ids_dev,
                           const uint8_t *starts_dev, int64_t n_envs, int64_t ring_rows, const int64_t *index_dev,
                           int64_t n_samples, const uint8_t *terminal_rows_dev, void *image_dev, int image_f32,
                           void *direction_dev, int direction_f32, uint8_t *mission_dev, void *stream) {
    if (!h || !rows_dev || !mission_ids_dev || !starts_dev || !index_dev || !image_dev || !direction_dev ||
        !mission_dev || n_envs <= 0 || n_samples < 0 || ring_rows < 0)
        return fail(MGX_ERR_INVALID, "mgx_gather: bad argument");
    if (ring_rows > 0 && ring_rows < h->kp.n_stack)
        return fail(MGX_ERR_INVALID, "mgx_gather_ring: the ring must hold n_stack rows");
    const int K = h->kp.n_stack;
    if (K > GATHER_MAXK) return fail(MGX_ERR_INVALID, "mgx_gather: n_stack > 8");
    if (n_samples == 0) return MGX_OK;
    if (!image_f32 != !direction_f32) return fail(MGX_ERR_INVALID, "mgx_gather: image and direction share one dtype");
    const int64_t nblk = (n_samples + GATHER_TILE - 1) / GATHER_TILE;
#define MGX_GATHER(KK)                                                                                           \
    case KK:                                                                                                     \
        if (image_f32)                                                                                           \
            hipLaunchKernelGGL((mgx_gather_kernel<KK, true>), dim3((unsigned)nblk), dim3(256), 0, (hipStream_t)stream, \
                               rows_dev, mission_ids_dev, starts_dev, n_envs, ring_rows, index_dev, n_samples, terminal_rows_dev, \
                               h->kp.mtok, image_dev, direction_dev, mission_dev);                              \
        else                                                                                                     \
            hipLaunchKernelGGL((mgx_gather_kernel<KK, false>), dim3((unsigned)nblk), dim3(256), 0, (hipStream_t)stream, \
                               rows_dev, mission_ids_dev, starts_dev, n_envs, ring_rows, index_dev, n_samples, terminal_rows_dev, \
                               h->kp.mtok, image_dev, direction_dev, mission_dev);                              \
        break;
    switch (K) {
        MGX_GATHER(1) MGX_GATHER(2) MGX_GATHER(3) MGX_GATHER(4) MGX_GATHER(5) MGX_GATHER(6) MGX_GATHER(7) MGX_GATHER(8)
        default: return fail(MGX_ERR_INVALID, "mgx_gather: n_stack out of range");
    }
#undef MGX_GATHER
    HIP_TRY(hipGetLastError());
    return MGX_OK;
}

mgx_status mgx_scene(mgx_handle *h, int64_t env, uint32_t *record, void *stream) {
    if (!h || !record) return fail(MGX_ERR_INVALID, "mgx_scene: null argument");
    if (env < 0 || env >= h->kp.n) return fail(MGX_ERR_INVALID, "mgx_scene: env out of range");
    if (!h->kp.start_rng) return fail(MGX_ERR_INVALID, "mgx_scene: needs inline resets (ring_depth = -1)");
    if (h->kp.S * h->kp.S > 4 * (MGX_SCENE_WORDS - 8 - MAX_OBJS)) return fail(MGX_ERR_INVALID, "mgx_scene: grid too large");
    uint32_t *dev = h->scene_dev;                 // handle-owned record (inline mode allocates it)
    HIP_TRY(hipMemsetAsync(dev, 0, MGX_SCENE_WORDS * sizeof(uint32_t), (hipStream_t)stream));
    MGX_GEN_LAUNCH(mgx_scene_kernel, dim3(1), dim3(64), h->lds_refill, (hipStream_t)stream, h->kp, env, dev);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(record, dev, MGX_SCENE_WORDS * sizeof(uint32_t), hipMemcpyDeviceToHost, (hipStream_t)stream));
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    return MGX_OK;
}

// Per-call shard scratch: the caller's (stats_scratch_dev) or the library's device-global one.
static double *gae_scratch(double *stats_scratch_dev) {
    if (stats_scratch_dev) return stats_scratch_dev;
    void *p = nullptr;
    (void)hipGetSymbolAddress(&p, HIP_SYMBOL(g_gae_shard));
    return static_cast<double *>(p);
}

mgx_status mgx_set_random_policy(mgx_handle *h, int enable, uint64_t seed) {
    if (!h) return fail(MGX_ERR_INVALID, "null handle");
    (void)hipSetDevice(h->device);
    if (!enable) {
        h->kp.rnd_ctr = nullptr;
        return MGX_OK;
    }
    const size_t words = (size_t)((h->kp.n + 31) / 32) + 1;   // one per rollout workgroup (32- or 64-env blocks)
    if (!h->allocs[17]) HIP_TRY(hipMalloc(&h->allocs[17], words * sizeof(unsigned long long)));
    HIP_TRY(hipMemset(h->allocs[17], 0, words * sizeof(unsigned long long)));
    HIP_TRY(hipDeviceSynchronize());
    h->kp.rnd_ctr = (unsigned long long *)h->allocs[17];
    h->kp.rnd_seed = seed;
    return MGX_OK;
}

mgx_status mgx_random_actions(int32_t *out_dev, int64_t count, int n_actions, uint64_t seed, uint64_t *counter_dev,
                              void *stream) {
    if (!out_dev || !counter_dev || count <= 0 || n_actions < 1 || n_actions > 65536)
        return fail(MGX_ERR_INVALID, "mgx_random_actions: bad argument");
    const int64_t blocks = std::min<int64_t>((count + 1023) / 1024, 1024);
    hipLaunchKernelGGL(mgx_random_actions_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, out_dev,
                       count, (uint32_t)n_actions, seed, (unsigned long long *)counter_dev);
    HIP_TRY(hipGetLastError());
    return MGX_OK;
}

mgx_status mgx_gae(const float *rewards_dev, const float *values_dev, const float *episode_starts_dev,
                   const float *last_values_dev, const uint8_t *last_dones_dev, int64_t T, int64_t N, float gamma,
                   float gamma_lambda, float *advantages_dev, float *returns_dev, double *adv_stats_dev,
                   double *stats_scratch_dev, void *stream) {
    if (!rewards_dev || !values_dev || !episode_starts_dev || !last_values_dev || !last_dones_dev ||
        !advantages_dev || !returns_dev || T <= 0 || N <= 0)
        return fail(MGX_ERR_INVALID, "mgx_gae: bad argument");
    double *shard = adv_stats_dev ? gae_scratch(stats_scratch_dev) : nullptr;
    if (adv_stats_dev && !shard) return fail(MGX_ERR_HIP, "mgx_gae: no shard scratch");
    const int64_t nblk = (N + 63) / 64;
    hipLaunchKernelGGL(mgx_gae_kernel<false>, dim3((unsigned)nblk), dim3(256), 0, (hipStream_t)stream, rewards_dev,
                       values_dev, (const void *)episode_starts_dev, last_values_dev, last_dones_dev, T, N, gamma,
                       gamma_lambda, advantages_dev, returns_dev, adv_stats_dev, shard);
    HIP_TRY(hipGetLastError());
    if (adv_stats_dev) {
        hipLaunchKernelGGL(mgx_gae_reduce_kernel, dim3(1), dim3(GAE_SHARDS), 0, (hipStream_t)stream, adv_stats_dev,
                           shard, (double)T * (double)N);
        HIP_TRY(hipGetLastError());
    }
    return MGX_OK;
}

mgx_status mgx_gae_dones(const float *rewards_dev, const float *values_dev, const uint8_t *dones_dev,
                         const float *last_values_dev, int64_t T, int64_t N, float gamma, float gamma_lambda,
                         float *advantages_dev, float *returns_dev, double *adv_stats_dev, double *stats_scratch_dev,
                         void *stream) {
    if (!rewards_dev || !values_dev || !dones_dev || !last_values_dev || !advantages_dev || !returns_dev || T <= 0 ||
        N <= 0)
        return fail(MGX_ERR_INVALID, "mgx_gae_dones: bad argument");
    double *shard = adv_stats_dev ? gae_scratch(stats_scratch_dev) : nullptr;
    if (adv_stats_dev && !shard) return fail(MGX_ERR_HIP, "mgx_gae_dones: no shard scratch");
    const int64_t nblk = (N + 63) / 64;
    hipLaunchKernelGGL(mgx_gae_kernel<true>, dim3((unsigned)nblk), dim3(256), 0, (hipStream_t)stream, rewards_dev,
                       values_dev, (const void *)dones_dev, last_values_dev, (const uint8_t *)nullptr, T, N, gamma,
                       gamma_lambda, advantages_dev, returns_dev, adv_stats_dev, shard);
    HIP_TRY(hipGetLastError());
    if (adv_stats_dev) {
        hipLaunchKernelGGL(mgx_gae_reduce_kernel, dim3(1), dim3(GAE_SHARDS), 0, (hipStream_t)stream, adv_stats_dev,
                           shard, (double)T * (double)N);
        HIP_TRY(hipGetLastError());
    }
    return MGX_OK;
}

mgx_status mgx_poll_error(mgx_handle *h, void *stream, uint32_t *bits) {
    if (!h || !bits) return fail(MGX_ERR_INVALID, "null argument");
    HIP_TRY(hipStreamSynchronize(h->side));
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    HIP_TRY(hipMemcpy(bits, h->kp.err, 4, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemset(h->kp.err, 0, 4));
    return MGX_OK;
}

mgx_status mgx_stats(mgx_handle *h, void *stream, uint64_t out[8]) {
    if (!h || !out) return fail(MGX_ERR_INVALID, "null argument");
    HIP_TRY(hipStreamSynchronize(h->side));
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    std::vector<ulonglong4> b((size_t)6 * h->kp.nblk);
    HIP_TRY(hipMemcpy(b.data(), h->kp.blk, b.size() * sizeof(ulonglong4), hipMemcpyDeviceToHost));
    uint64_t c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // blk sections: [0, nblk) step kernel (x steps, y resets), [nblk, 2 nblk) fixup, [2 nblk, 6 nblk)
    // refill (x: that wave's consumption at its last launch, not a counter); z live-locks and w max MT cursor
    // in every section
    for (size_t i = 0; i < b.size(); i++) {
        const ulonglong4 &v = b[i];
        if (i < (size_t)2 * h->kp.nblk) c[0] += v.x;
        c[1] += v.y; c[2] += v.z; c[3] = v.w > c[3] ? v.w : c[3];
    }
    if (h->kp.D > 0) {   // episodes queued in the rings: sum of (tail - head) mod 2^16
        std::vector<rpos_t> ht((size_t)2 * h->kp.n);
        HIP_TRY(hipMemcpy(ht.data(), h->kp.ring_head, ht.size() * sizeof(rpos_t), hipMemcpyDeviceToHost));
        for (int64_t i = 0; i < h->kp.n; i++) c[4] += (rpos_t)(ht[(size_t)(h->kp.n + i)] - ht[(size_t)i]);
    }
    c[5] = h->refill_launches;
    c[6] = h->calls;
    {
        MtCtl m;
        HIP_TRY(hipMemcpy(&m, h->kp.mtc, 16, hipMemcpyDeviceToHost));   // lo, hi
        c[7] = m.hi * (uint64_t)MT_FIELDS;
    }
    for (int i = 0; i < 8; i++) out[i] = c[i];
    return MGX_OK;
}

mgx_status mgx_ring_levels(mgx_handle *h, void *stream, uint16_t *levels) {
    if (!h || !levels) return fail(MGX_ERR_INVALID, "null argument");
    HIP_TRY(hipStreamSynchronize(h->side));
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    const int64_t N = h->kp.n;
    if (h->kp.D <= 0) {
        std::memset(levels, 0, (size_t)N * sizeof(uint16_t));
        return MGX_OK;
    }
    std::vector<rpos_t> ht((size_t)2 * N);
    HIP_TRY(hipMemcpy(ht.data(), h->kp.ring_head, ht.size() * sizeof(rpos_t), hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < N; i++) levels[i] = (rpos_t)(ht[(size_t)(N + i)] - ht[(size_t)i]);
    return MGX_OK;
}

mgx_status mgx_dump_state(mgx_handle *h, void *stream, uint8_t *grid, uint8_t *agent, uint8_t *carrying,
                          int32_t *step_count, uint8_t *mission_done, double *stored_reward, int64_t *mt_words,
                          uint64_t *pcg, uint8_t *target, uint8_t *mission_id) {
    if (!h) return fail(MGX_ERR_INVALID, "null handle");
    HIP_TRY(hipStreamSynchronize(h->side));
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    const int64_t N = h->kp.n;
    const int S = h->kp.S, GS = h->kp.GS;
    std::vector<EnvState> st((size_t)N);
    HIP_TRY(hipMemcpy(st.data(), h->kp.state, (size_t)N * sizeof(EnvState), hipMemcpyDeviceToHost));
    auto enc = [](uint8_t code, uint8_t *o4) {
        int t = code & 15, c = (code >> 4) & 7, a = code >> 7;
        int s = t == T_DOOR ? 1 + a : 0;
        if (t == T_OPEN) t = T_DOOR;
        o4[0] = (uint8_t)t; o4[1] = (uint8_t)c; o4[2] = (uint8_t)s; o4[3] = (uint8_t)(t == T_BOX && a);
    };
    if (grid) {
        std::vector<uint8_t> g((size_t)N * GS);
        HIP_TRY(hipMemcpy(g.data(), h->kp.grid, g.size(), hipMemcpyDeviceToHost));
        for (int64_t i = 0; i < N; i++)
            for (int x = 0; x < S; x++)
                for (int y = 0; y < S; y++) enc(g[(size_t)i * GS + y * S + x], grid + (((size_t)i * S + x) * S + y) * 4);
    }
    std::vector<uint4> pc, cr;
    if (pcg || mt_words) {
        pc.resize((size_t)N * 2);
        cr.resize((size_t)N * 2);
        HIP_TRY(hipMemcpy(pc.data(), h->kp.pcg, pc.size() * 16, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(cr.data(), h->kp.cur_rng, cr.size() * 16, hipMemcpyDeviceToHost));
    }
    const int ms = S * S;
    for (int64_t i = 0; i < N; i++) {
        const EnvState &s = st[(size_t)i];
        if (agent) { agent[i * 3] = s.ax; agent[i * 3 + 1] = s.ay; agent[i * 3 + 2] = s.dir; }
        if (carrying) {
            if (s.carry == 0) std::memset(carrying + i * 4, 0, 4);
            else enc(s.carry, carrying + i * 4);
        }
        if (step_count) step_count[i] = s.step_count;
        if (mission_done) mission_done[i] = s.mission_done;
        if (stored_reward) stored_reward[i] = s.reward_step < 0 ? NAN : 1.0 - 0.9 * ((double)s.reward_step / (double)ms);
        if (mt_words) mt_words[i] = (int64_t)((uint64_t)cr[(size_t)i * 2 + 1].z | ((uint64_t)cr[(size_t)i * 2 + 1].w << 32));
        if (pcg) {
            const uint4 a = cr[(size_t)i * 2], b = pc[(size_t)i * 2 + 1], c = cr[(size_t)i * 2 + 1];
            uint64_t *o6 = pcg + i * 6;
            o6[0] = ((uint64_t)a.x << 32) | a.y; o6[1] = ((uint64_t)a.z << 32) | a.w;
            o6[2] = ((uint64_t)b.x << 32) | b.y; o6[3] = ((uint64_t)b.z << 32) | b.w;
            o6[4] = c.y; o6[5] = c.x;
        }
        if (target) { target[i * 3] = s.tx; target[i * 3 + 1] = s.ty; target[i * 3 + 2] = s.target_action; }
        if (mission_id) mission_id[i] = s.mission_id;
    }
    return MGX_OK;
}

}  // extern "C"
