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
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/mgx.h"
#include "mgx_device.h"

using namespace mgx;

namespace {

constexpr int BLOCK_ENVS = 64;
constexpr int BLOCK_THREADS = 256;
constexpr int FRAME = 147;                 // 3 x 7 x 7
constexpr int SCRATCH_PER_ENV = WIN_STRIDE * 4 + OBJ_STRIDE * 4;   // LDS bytes per resetting lane

struct KParams {
    EnvState *state;
    uint8_t *grid;
    uint4 *pcg;        // [N][2]
    uint4 *aux;        // [N]
    const uint32_t *mt;
    const uint8_t *mtok;
    unsigned long long *counters;   // [0] steps [1] resets [2] livelocks [3] max cursor
    uint32_t *err;
    uint64_t tlen;
    int64_t n;
    int64_t seed_base;              // base_seed + env_index_offset
    int S, GS, GSL, n_stack, img_bytes, stk_lds, problem, cfg_mission, num_objects, all_doors_open;
    uint32_t llw;
    int terminal_mode, mission64;
};

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

__device__ __forceinline__ void load_gen(Gen &G, const KParams &p, int64_t e, uint8_t *g, uint8_t *scratch, int lane) {
    G.g = g;
    G.S = p.S;
    G.table = p.mt;
    G.tlen = p.tlen;
    G.win = reinterpret_cast<uint32_t *>(scratch + lane * (WIN_STRIDE * 4));
    G.objs = reinterpret_cast<uint32_t *>(scratch + BLOCK_ENVS * (WIN_STRIDE * 4) + lane * (OBJ_STRIDE * 4));
    G.llw = p.llw;
    G.err = 0;
    G.problem = p.problem;
    G.cfg_mission = p.cfg_mission;
    G.num_objects = p.num_objects;
    G.all_doors_open = p.all_doors_open;
    G.abort = false;
    G.nobjs = 0;
    G.ax = G.ay = -1;
    G.adir = 0;
}

__device__ __forceinline__ void load_rng(Gen &G, const KParams &p, int64_t e) {
    uint4 s = p.pcg[2 * e], i = p.pcg[2 * e + 1], a = p.aux[e];
    G.pcg.sh = ((uint64_t)s.x << 32) | s.y;
    G.pcg.sl = ((uint64_t)s.z << 32) | s.w;
    G.pcg.ih = ((uint64_t)i.x << 32) | i.y;
    G.pcg.il = ((uint64_t)i.z << 32) | i.w;
    G.pcg.uinteger = a.x;
    G.pcg.has = a.y;
    G.cur = (uint64_t)a.z | ((uint64_t)a.w << 32);
    G.wbase = ~0ull >> 1;   // empty window
}
__device__ __forceinline__ void store_rng(const Gen &G, const KParams &p, int64_t e) {
    p.pcg[2 * e] = make_uint4((uint32_t)(G.pcg.sh >> 32), (uint32_t)G.pcg.sh, (uint32_t)(G.pcg.sl >> 32), (uint32_t)G.pcg.sl);
    p.pcg[2 * e + 1] = make_uint4((uint32_t)(G.pcg.ih >> 32), (uint32_t)G.pcg.ih, (uint32_t)(G.pcg.il >> 32), (uint32_t)G.pcg.il);
    p.aux[e] = make_uint4(G.pcg.uinteger, G.pcg.has, (uint32_t)G.cur, (uint32_t)(G.cur >> 32));
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
}

// ============================================================== reset kernel
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
        Gen G;
        load_gen(G, p, e, s_grid + tid * p.GSL, s_scr, tid);
        pcg_seed(G.pcg, (uint64_t)(p.seed_base + e));   // gymnasium Env.reset(seed=seed+i)
        G.cur = 0;                                       // random.seed(cfg.seed) in every worker
        G.wbase = ~0ull >> 1;
        ResetOut R;
        reset_env(G, R);
        EnvState st;
        st.ax = (uint8_t)G.ax; st.ay = (uint8_t)G.ay; st.dir = (uint8_t)G.adir; st.carry = 0;
        st.step_count = 0; st.reward_step = -1;
        st.tx = R.tx; st.ty = R.ty; st.target_action = R.ta; st.mission_id = R.mission_id;
        st.mission_done = 0; st.frames = 1; st.flags = 0; st.pad = 0;
        p.state[e] = st;
        store_rng(G, p, e);
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
        atomicAdd(&p.counters[1], (unsigned long long)ne);
        atomicAdd(&p.counters[2], s_ll);
        atomicMax(&p.counters[3], s_maxcur);
        if (s_err) atomicOr(p.err, s_err);
    }
}

// =============================================================== step kernel
template <typename ActT>
__global__ __launch_bounds__(BLOCK_THREADS) void mgx_step_kernel(KParams p, KOut o, const ActT *__restrict__ actions) {
    extern __shared__ __align__(16) uint8_t smem[];
    uint8_t *s_stk = smem;                       // image stacks [64][img_bytes]; later reset scratch
    uint8_t *s_grid = smem + p.stk_lds;          // grids [64][GSL]
    __shared__ uint8_t s_done[BLOCK_ENVS];
    __shared__ uint8_t s_dirty[BLOCK_ENVS];
    __shared__ uint8_t s_term_out[BLOCK_ENVS];   // write terminal image stack
    __shared__ unsigned long long s_ndone, s_ll, s_maxcur;
    __shared__ uint32_t s_err;

    const int tid = threadIdx.x;
    const int64_t e0 = (int64_t)blockIdx.x * BLOCK_ENVS;
    const int ne = (int)min<int64_t>(BLOCK_ENVS, p.n - e0);
    const int IMG = p.img_bytes;
    if (tid == 0) { s_ndone = 0; s_ll = 0; s_maxcur = 0; s_err = 0; }
#ifdef MGX_STAMPS
    const unsigned long long ts0 = __builtin_amdgcn_s_memtime();
    unsigned long long ts1 = 0, ts2 = 0, ts3 = 0;
#endif

    // ---- phase 1: stage grids + image stacks (slot 0 of each env is dead: skip it)
    grid_copy_in(s_grid, p.grid + e0 * p.GS, ne, p.GS, p.GSL);
    {
        const uint8_t *gimg = o.img + e0 * (int64_t)IMG;
        const int nbytes = ne * IMG;
        const int n16 = nbytes >> 4;
        const uint4 *src = reinterpret_cast<const uint4 *>(gimg);
        uint4 *dst = reinterpret_cast<uint4 *>(s_stk);
        for (int i = tid; i < n16; i += BLOCK_THREADS) {
            int b0 = i << 4;
            int off = b0 % IMG;
            // chunk entirely inside slot 0 of one env -> not needed
            if (off + 16 <= FRAME) continue;
            dst[i] = src[i];
        }
        for (int i = (n16 << 4) + tid; i < nbytes; i += BLOCK_THREADS) s_stk[i] = gimg[i];
    }
    __syncthreads();

    // ---- phase 2: one lane per env: MiniGridEnv.step + PlaygroundEnv.step
    EnvState st;
    bool done = false;
    uint32_t my_err = 0;
    if (tid < ne) {
        const int64_t e = e0 + tid;
        st = p.state[e];
        int a = (int)actions[e];
        if ((unsigned)a > 6u) { my_err |= MGX_DEVERR_BAD_ACTION; a = -1; }
        uint8_t *g = s_grid + tid * p.GSL;
        const int S = p.S, ms = S * S;
        const int sc = st.step_count + 1;
        int ax = st.ax, ay = st.ay, dir = st.dir;
        uint8_t carry = st.carry;
        const int fx = ax + ((dir == 0) - (dir == 2)), fy = ay + ((dir == 1) - (dir == 3));
        uint8_t *fp = g + fy * S + fx;
        const uint8_t fc = *fp;
        const int ft = fc & 15;
        bool term = false, dirty = false;
        double rew = 0.0;
        switch (a) {                                   // MiniGridEnv.step (3P)
            case A_LEFT: dir = (dir + 3) & 3; break;
            case A_RIGHT: dir = (dir + 1) & 3; break;
            case A_FORWARD:
                if (can_overlap(fc)) { ax = fx; ay = fy; }
                if (ft == T_GOAL) { term = true; rew = reward_at(sc, ms); }
                if (ft == T_LAVA) term = true;
                break;
            case A_PICKUP:
                if (can_pickup(fc) && carry == 0) { carry = fc; *fp = CODE_EMPTY; dirty = true; }
                break;
            case A_DROP:
                if (ft == T_EMPTY && carry != 0) { *fp = carry; carry = 0; dirty = true; }
                break;
            case A_TOGGLE:
                if (ft == T_DOOR) {
                    if (fc >> 7) {                     // locked
                        if ((carry & 15) == T_KEY && ((carry >> 4) & 7) == ((fc >> 4) & 7)) {
                            *fp = mk_code(T_OPEN, (fc >> 4) & 7, 0); dirty = true;
                        }
                    } else { *fp = mk_code(T_OPEN, (fc >> 4) & 7, 0); dirty = true; }
                } else if (ft == T_OPEN) {
                    *fp = mk_code(T_DOOR, (fc >> 4) & 7, 0); dirty = true;
                } else if (ft == T_BOX) {
                    *fp = (fc >> 7) ? mk_code(T_KEY, (fc >> 4) & 7, 0) : CODE_EMPTY; dirty = true;
                }
                break;
            default: break;                            // done (and invalid) -> no-op
        }
        const bool trunc = sc >= ms;
        // gen_obs() happens here, before PlaygroundEnv's key consumption (Q3)
        uint8_t *fr = s_stk + tid * IMG;               // dead slot 0 -> rotated to newest below
        render_view(g, S, ax, ay, dir, carry, [&](int k, uint32_t v) {
            fr[k] = (uint8_t)v;
            fr[49 + k] = (uint8_t)(v >> 8);
            fr[98 + k] = (uint8_t)(v >> 16);
        });
        // ---- PlaygroundEnv.step (custom_env.py:269-330)
        int mdone = st.mission_done, rs = st.reward_step;
        const bool is_gtg = st.mission_id == CMD_GOTOGOAL;
        if (term) {
            if (!is_gtg) { mdone = 0; rs = -1; rew = 0.0; }
        } else {
            if (a == A_TOGGLE) {
                const uint8_t f2 = *fp;
                if (is_door(f2) && carry != 0 && ((f2 >> 4) & 7) == ((carry >> 4) & 7)) carry = 0;  // Q4
            }
            if (!mdone) {
                const bool has_t = st.tx != NONE8;
                bool arrived = false;
                if (has_t) {
                    if (st.target_action != NONE8 && st.target_action != 0) {
                        const int nfx = ax + ((dir == 0) - (dir == 2)), nfy = ay + ((dir == 1) - (dir == 3));
                        arrived = nfx == st.tx && nfy == st.ty;
                    } else if (ax == st.tx && ay == st.ty) {
                        if (rs < 0) rs = sc;
                        mdone = 1;
                    }
                }
                if (arrived && a == (int)st.target_action) { if (rs < 0) rs = sc; mdone = 1; }
                if (!has_t && st.target_action != NONE8 && a == (int)st.target_action) { if (rs < 0) rs = sc; mdone = 1; }
            }
            if (a == A_DONE) {
                rew = mdone ? reward_at(rs, ms) : 0.0;    // stored self.reward, or 0 (not manual)
                mdone = 0; rs = -1; term = true;
            }
        }
        done = term || trunc;
        o.reward[e] = (float)rew;
        if (o.reward64) o.reward64[e] = rew;
        o.term[e] = term;
        o.trunc[e] = trunc;
        if (o.done) o.done[e] = done;
        if (o.ep_ret) o.ep_ret[e] = (float)rew;       // only the final step can pay a reward
        if (o.ep_len) o.ep_len[e] = sc;
        if (o.livelock) o.livelock[e] = 0;
        const bool want_term = done && (p.terminal_mode == MGX_TERMINAL_ALL ||
                                        (p.terminal_mode == MGX_TERMINAL_TRUNCATED && trunc && !term));
        const int frames = min((int)st.frames + 1, p.n_stack);
        const uint8_t *tok = p.mtok + st.mission_id * 32;
        if (!done) {
            dir_stack_roll(o.dir, o.dir, e, p.n_stack, dir);
            if (st.frames < p.n_stack)                 // stack still filling: one slot flips 0 -> mission
                write_mission_slot(o.mis, p.mission64, e, p.n_stack, p.n_stack - frames, tok);
            st.ax = (uint8_t)ax; st.ay = (uint8_t)ay; st.dir = (uint8_t)dir; st.carry = carry;
            st.step_count = (uint16_t)sc; st.reward_step = (int16_t)rs; st.mission_done = (uint8_t)mdone;
            st.frames = (uint8_t)frames;
            p.state[e] = st;
        } else {
            if (want_term) {
                dir_stack_roll(o.dir, o.t_dir, e, p.n_stack, dir);
                write_mission_stack(o.t_mis, p.mission64, e, p.n_stack, frames, tok);
            }
            // survives the reset (Q2): mission_done / stored reward
            st.reward_step = (int16_t)rs; st.mission_done = (uint8_t)mdone;
        }
        s_done[tid] = done;
        s_dirty[tid] = dirty;
        s_term_out[tid] = want_term;
        if (done) atomicAdd(&s_ndone, 1ull);
    } else if (tid < BLOCK_ENVS) {
        s_done[tid] = 0; s_dirty[tid] = 0; s_term_out[tid] = 0;
    }
    __syncthreads();
#ifdef MGX_STAMPS
    ts1 = __builtin_amdgcn_s_memtime();
#endif

    // ---- phase 3: write the rolled image stacks (newest frame sits in slot 0 of LDS)
    {
        uint8_t *gimg = o.img + e0 * (int64_t)IMG;
        if ((IMG & 3) == 0) {
            // dword path (n_stack % 4 == 0): out byte o = lds[(o + 147) mod IMG]
            //   -> out dword j = alignbyte(dw[(j+37) mod DW], dw[(j+36) mod DW], 3)
            const int DW = IMG >> 2;
            const uint32_t *s32 = reinterpret_cast<const uint32_t *>(s_stk);
            uint32_t *g32 = reinterpret_cast<uint32_t *>(gimg);
            for (int k = tid; k < ne * DW; k += BLOCK_THREADS) {
                const int e = k / DW, j = k - e * DW;
                uint32_t out = 0;
                if (!s_done[e]) {
                    int j0 = j + FRAME / 4;
                    if (j0 >= DW) j0 -= DW;
                    const int j1 = (j0 + 1 == DW) ? 0 : j0 + 1;
                    out = __builtin_amdgcn_alignbyte(s32[e * DW + j1], s32[e * DW + j0], FRAME & 3);
                }
                g32[k] = out;
            }
        } else {
            const int nbytes = ne * IMG;
            for (int b = tid; b < nbytes; b += BLOCK_THREADS) {
                const int e = b / IMG, off = b - e * IMG;
                int src = off + FRAME;
                if (src >= IMG) src -= IMG;
                gimg[b] = s_done[e] ? 0 : s_stk[e * IMG + src];
            }
        }
        // terminal stacks (rare: done envs that asked for one)
        if (p.terminal_mode != MGX_TERMINAL_NONE && s_ndone) {
            for (int le = 0; le < ne; le++) {
                if (!s_term_out[le]) continue;
                uint8_t *dst = o.t_img + (e0 + le) * (int64_t)IMG;
                for (int off = tid; off < IMG; off += BLOCK_THREADS) {
                    int src = off + FRAME;
                    if (src >= IMG) src -= IMG;
                    dst[off] = s_stk[le * IMG + src];
                }
            }
        }
    }
    __syncthreads();
#ifdef MGX_STAMPS
    ts2 = __builtin_amdgcn_s_memtime();
#endif

    // ---- phase 4: fused auto-reset of done envs (SubprocVecEnv: env.reset() unseeded)
    if (s_ndone) {
        if (tid < ne && done) {
            const int64_t e = e0 + tid;
            Gen G;
            load_gen(G, p, e, s_grid + tid * p.GSL, s_stk, tid);
            load_rng(G, p, e);
            ResetOut R;
            reset_env(G, R);
            EnvState ns;
            ns.ax = (uint8_t)G.ax; ns.ay = (uint8_t)G.ay; ns.dir = (uint8_t)G.adir; ns.carry = 0;
            ns.step_count = 0; ns.reward_step = st.reward_step;
            ns.tx = R.tx; ns.ty = R.ty; ns.target_action = R.ta; ns.mission_id = R.mission_id;
            ns.mission_done = st.mission_done; ns.frames = 1; ns.flags = 0; ns.pad = 0;
            p.state[e] = ns;
            store_rng(G, p, e);
            write_fresh_frame(p, o.img, e, G.g, G.ax, G.ay, G.adir);
            dir_stack_fresh(o.dir, e, p.n_stack, G.adir);
            write_mission_stack(o.mis, p.mission64, e, p.n_stack, 1, p.mtok + R.mission_id * 32);
            if (o.livelock) o.livelock[e] = R.livelocks;
            s_dirty[tid] = 1;
            atomicAdd(&s_ll, (unsigned long long)R.livelocks);
            atomicMax(&s_maxcur, (unsigned long long)G.cur);
            my_err |= G.err;
        }
        __syncthreads();
    }
    if (my_err) atomicOr(&s_err, my_err);
#ifdef MGX_STAMPS
    ts3 = __builtin_amdgcn_s_memtime();
#endif

    // ---- phase 5: write back grids that changed
    grid_copy_out(p.grid + e0 * p.GS, s_grid, ne, p.GS, p.GSL, s_dirty);
    __syncthreads();
    if (tid == 0) {
        atomicAdd(&p.counters[0], (unsigned long long)ne);
        if (s_ndone) {
            atomicAdd(&p.counters[1], s_ndone);
            atomicAdd(&p.counters[2], s_ll);
            atomicMax(&p.counters[3], s_maxcur);
        }
        if (s_err) atomicOr(p.err, s_err);
#ifdef MGX_STAMPS
        const unsigned long long ts4 = __builtin_amdgcn_s_memtime();
        atomicAdd(&p.counters[4], ts1 - ts0);   // phase 1+2: stage + step logic
        atomicAdd(&p.counters[5], ts2 - ts1);   // phase 3: stack roll write-back
        atomicAdd(&p.counters[6], ts3 - ts2);   // phase 4: fused resets
        atomicAdd(&p.counters[7], ts4 - ts3);   // phase 5: grid write-back
#endif
    }
}

// ================================================================ GAE kernel
// DictRolloutBuffer.compute_returns_and_advantage (SB3; fp32, numpy op order,
// built with -ffp-contract=off):  delta = ((r + (g*nv)*nnt) - V);  last = delta + (c*nnt)*last
__global__ __launch_bounds__(256) void mgx_gae_kernel(const float *__restrict__ r, const float *__restrict__ v,
                                                      const float *__restrict__ es, const float *__restrict__ lv,
                                                      const uint8_t *__restrict__ ld, int64_t T, int64_t N, float g,
                                                      float c, float *__restrict__ adv, float *__restrict__ ret,
                                                      double *__restrict__ stats) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double s1 = 0.0, s2 = 0.0;
    if (i < N) {
        float last = 0.0f;
        float nnt = 1.0f - (float)ld[i];
        float nv = lv[i];
        for (int64_t t = T - 1; t >= 0; --t) {
            const int64_t k = t * N + i;
            const float vt = v[k];
            const float rt = r[k];
            const float est = es[k];
            const float delta = (rt + (g * nv) * nnt) - vt;
            last = delta + (c * nnt) * last;
            adv[k] = last;
            ret[k] = last + vt;
            s1 += (double)last;
            s2 += (double)last * (double)last;
            nnt = 1.0f - est;       // for step t-1: 1 - episode_starts[t]
            nv = vt;
        }
    }
    if (stats) {
        __shared__ double red[2][256 / 64];
        for (int off = 32; off > 0; off >>= 1) {
            s1 += __shfl_down(s1, off);
            s2 += __shfl_down(s2, off);
        }
        const int w = threadIdx.x >> 6;
        if ((threadIdx.x & 63) == 0) { red[0][w] = s1; red[1][w] = s2; }
        __syncthreads();
        if (threadIdx.x == 0) {
            double a = 0, b = 0;
            for (int k = 0; k < (int)(blockDim.x >> 6); k++) { a += red[0][k]; b += red[1][k]; }
            int64_t cnt = min<int64_t>(blockDim.x, N - (int64_t)blockIdx.x * blockDim.x) * T;
            atomicAdd(&stats[0], a);
            atomicAdd(&stats[1], b);
            atomicAdd(&stats[2], (double)cnt);
        }
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

bool mission_text(int id, std::string &out) {
    if (id < 0 || id > 255) return false;
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
    size_t lds_step, lds_reset;
    void *allocs[8];
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

static mgx_status validate(const mgx_config *c) {
    if (!c) return fail(MGX_ERR_INVALID, "null config");
    if (c->size < 5 || c->size > 16) return fail(MGX_ERR_INVALID, "size must be in 5..16");
    if (c->n_envs <= 0) return fail(MGX_ERR_INVALID, "n_envs must be > 0");
    if (c->n_stack < 1 || c->n_stack > 8) return fail(MGX_ERR_INVALID, "n_stack must be in 1..8");
    if (!c->see_through_walls) return fail(MGX_ERR_INVALID, "see_through_walls=false (process_vis) is not supported");
    if (c->obstacles) return fail(MGX_ERR_INVALID, "obstacles=true is not supported");
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
        case MGX_PROBLEM_FULL: case MGX_PROBLEM_DRP: case MGX_PROBLEM_MOV:
            return fail(MGX_ERR_INVALID, "problem full/drp/mov is not built yet (DESIGN.md, next)");
        default:
            return fail(MGX_ERR_INVALID, "Invalid problem type given");
    }
    if (c->num_objects < 0) return fail(MGX_ERR_INVALID, "num_objects must be >= 0");
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
    if (h->cfg.mt_table_words <= 0) h->cfg.mt_table_words = (int64_t)1 << 24;
    h->cfg.mt_table_words = (h->cfg.mt_table_words + 3) & ~(int64_t)3;
    const int64_t N = cfg->n_envs;
    const int S = cfg->size;
    const int GS = ((S * S) + 15) & ~15;
    const int IMG = FRAME * cfg->n_stack;
    const int64_t tlen = h->cfg.mt_table_words;

    auto bail = [&](mgx_status st) {
        for (void *&p : h->allocs) if (p) { (void)hipFree(p); p = nullptr; }
        delete h;
        (void)hipSetDevice(prev);
        return st;
    };
    size_t sizes[6] = {(size_t)N * sizeof(EnvState), (size_t)N * GS, (size_t)N * 32, (size_t)N * 16,
                       (size_t)(tlen + MT_WIN + 4) * 4, 256 * 32 + 64};
    for (int i = 0; i < 6; i++) {
        hipError_t e = hipMalloc(&h->allocs[i], sizes[i]);
        if (e != hipSuccess) return bail(fail(MGX_ERR_OOM, std::string("hipMalloc: ") + hipGetErrorString(e)));
    }
    {
        hipError_t e = hipMalloc(&h->allocs[6], 8 * sizeof(unsigned long long) + 64);
        if (e != hipSuccess) return bail(fail(MGX_ERR_OOM, "hipMalloc counters"));
        e = hipMemset(h->allocs[6], 0, 8 * sizeof(unsigned long long) + 64);
        if (e != hipSuccess) return bail(fail(MGX_ERR_HIP, "hipMemset counters"));
    }
    // MT19937(base_seed) output table, zero-padded by one window
    {
        std::vector<uint32_t> tab((size_t)(tlen + MT_WIN + 4), 0u);
        HostMT m;
        m.seed((uint64_t)cfg->base_seed);
        for (int64_t i = 0; i < tlen; i++) tab[(size_t)i] = m.next();
        hipError_t e = hipMemcpy(h->allocs[4], tab.data(), tab.size() * 4, hipMemcpyHostToDevice);
        if (e != hipSuccess) return bail(fail(MGX_ERR_HIP, "upload MT table"));
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
    p.mt = (const uint32_t *)h->allocs[4];
    p.mtok = (const uint8_t *)h->allocs[5];
    p.counters = (unsigned long long *)h->allocs[6];
    p.err = (uint32_t *)((char *)h->allocs[6] + 8 * sizeof(unsigned long long));
    p.tlen = (uint64_t)tlen;
    p.n = N;
    p.seed_base = cfg->base_seed + cfg->env_index_offset;
    p.S = S;
    p.GS = GS;
    p.GSL = GS + 4;
    p.n_stack = cfg->n_stack;
    p.img_bytes = IMG;
    const int scratch = BLOCK_ENVS * SCRATCH_PER_ENV;
    p.stk_lds = (std::max(BLOCK_ENVS * IMG, scratch) + 15) & ~15;
    p.problem = cfg->problem;
    p.cfg_mission = cfg->mission;
    p.num_objects = cfg->num_objects;
    p.all_doors_open = cfg->all_doors_open;
    p.llw = (uint32_t)h->cfg.livelock_words;
    p.terminal_mode = cfg->terminal_mode;
    p.mission64 = cfg->mission_int64;
    h->lds_step = (size_t)p.stk_lds + (size_t)BLOCK_ENVS * (GS + 4);
    h->lds_reset = h->lds_step;
    HIP_TRY(hipFuncSetAttribute((const void *)mgx_step_kernel<int32_t>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_step));
    HIP_TRY(hipFuncSetAttribute((const void *)mgx_step_kernel<int64_t>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_step));
    HIP_TRY(hipFuncSetAttribute((const void *)mgx_reset_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds_reset));
    (void)hipSetDevice(prev);
    *out = h;
    return MGX_OK;
}

mgx_status mgx_destroy(mgx_handle *h) {
    if (!h) return MGX_OK;
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(h->device);
    for (void *&p : h->allocs) if (p) { (void)hipFree(p); p = nullptr; }
    (void)hipSetDevice(prev);
    delete h;
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
    const int64_t nblk = (h->kp.n + BLOCK_ENVS - 1) / BLOCK_ENVS;
    hipLaunchKernelGGL(mgx_reset_kernel, dim3((unsigned)nblk), dim3(BLOCK_THREADS), h->lds_reset,
                       (hipStream_t)stream, h->kp, o);
    HIP_TRY(hipGetLastError());
    return MGX_OK;
}

mgx_status mgx_step(mgx_handle *h, const void *actions_dev, int action_bytes, const mgx_step_out *out, void *stream) {
    if (!h || !out || !actions_dev) return fail(MGX_ERR_INVALID, "mgx_step: null argument");
    if (!out->obs.image_dev || !out->obs.direction_dev || !out->obs.mission_dev || !out->reward_dev ||
        !out->terminated_dev || !out->truncated_dev)
        return fail(MGX_ERR_INVALID, "mgx_step: missing output buffer");
    if (h->kp.terminal_mode != MGX_TERMINAL_NONE &&
        (!out->terminal.image_dev || !out->terminal.direction_dev || !out->terminal.mission_dev))
        return fail(MGX_ERR_INVALID, "mgx_step: terminal_mode needs terminal buffers");
    KOut o = make_out(nullptr, out);
    const int64_t nblk = (h->kp.n + BLOCK_ENVS - 1) / BLOCK_ENVS;
    if (action_bytes == 4)
        hipLaunchKernelGGL(mgx_step_kernel<int32_t>, dim3((unsigned)nblk), dim3(BLOCK_THREADS), h->lds_step,
                           (hipStream_t)stream, h->kp, o, (const int32_t *)actions_dev);
    else if (action_bytes == 8)
        hipLaunchKernelGGL(mgx_step_kernel<int64_t>, dim3((unsigned)nblk), dim3(BLOCK_THREADS), h->lds_step,
                           (hipStream_t)stream, h->kp, o, (const int64_t *)actions_dev);
    else
        return fail(MGX_ERR_INVALID, "action_bytes must be 4 or 8");
    HIP_TRY(hipGetLastError());
    return MGX_OK;
}

mgx_status mgx_gae(const float *rewards_dev, const float *values_dev, const float *episode_starts_dev,
                   const float *last_values_dev, const uint8_t *last_dones_dev, int64_t T, int64_t N, float gamma,
                   float gamma_lambda, float *advantages_dev, float *returns_dev, double *adv_stats_dev,
                   void *stream) {
    if (!rewards_dev || !values_dev || !episode_starts_dev || !last_values_dev || !last_dones_dev ||
        !advantages_dev || !returns_dev || T <= 0 || N <= 0)
        return fail(MGX_ERR_INVALID, "mgx_gae: bad argument");
    const int64_t nblk = (N + 255) / 256;
    hipLaunchKernelGGL(mgx_gae_kernel, dim3((unsigned)nblk), dim3(256), 0, (hipStream_t)stream, rewards_dev,
                       values_dev, episode_starts_dev, last_values_dev, last_dones_dev, T, N, gamma, gamma_lambda,
                       advantages_dev, returns_dev, adv_stats_dev);
    HIP_TRY(hipGetLastError());
    return MGX_OK;
}

mgx_status mgx_poll_error(mgx_handle *h, void *stream, uint32_t *bits) {
    if (!h || !bits) return fail(MGX_ERR_INVALID, "null argument");
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    HIP_TRY(hipMemcpy(bits, h->kp.err, 4, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemset(h->kp.err, 0, 4));
    return MGX_OK;
}

mgx_status mgx_stats(mgx_handle *h, void *stream, uint64_t out[4]) {
    if (!h || !out) return fail(MGX_ERR_INVALID, "null argument");
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    unsigned long long c[8];
    HIP_TRY(hipMemcpy(c, h->kp.counters, sizeof c, hipMemcpyDeviceToHost));
    for (int i = 0; i < 8; i++) out[i] = c[i];
    return MGX_OK;
}

mgx_status mgx_dump_state(mgx_handle *h, void *stream, uint8_t *grid, uint8_t *agent, uint8_t *carrying,
                          int32_t *step_count, uint8_t *mission_done, double *stored_reward, int64_t *mt_words,
                          uint64_t *pcg, uint8_t *target, uint8_t *mission_id) {
    if (!h) return fail(MGX_ERR_INVALID, "null handle");
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
    std::vector<uint4> pc, ax;
    if (pcg || mt_words) {
        pc.resize((size_t)N * 2);
        ax.resize((size_t)N);
        HIP_TRY(hipMemcpy(pc.data(), h->kp.pcg, pc.size() * 16, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(ax.data(), h->kp.aux, ax.size() * 16, hipMemcpyDeviceToHost));
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
        if (mt_words) mt_words[i] = (int64_t)((uint64_t)ax[(size_t)i].z | ((uint64_t)ax[(size_t)i].w << 32));
        if (pcg) {
            const uint4 a = pc[(size_t)i * 2], b = pc[(size_t)i * 2 + 1], c = ax[(size_t)i];
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
