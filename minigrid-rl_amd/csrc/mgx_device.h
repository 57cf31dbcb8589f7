// mgx_device.h -- device-side MiniGrid semantics for the MI355X engine.
//
// One env per lane.  Env grids are 1 byte per cell (code below), staged per
// workgroup in LDS; reset generation runs on the env's LDS grid slot with the
// shared MT19937 output table read through a per-lane LDS window.
//
// Reference behaviour reproduced (file:line into /root/reference):
//   PlaygroundEnv.step             src/custom_env.py:269-330   -> step_env()
//   PlaygroundEnv._gen_grid        src/custom_env.py:122-267   -> gen_attempt()/reset_env()
//   _generate_multi_map            src/custom_env.py:595-615   -> gen_multi()
//   _generate_2/3/4_rooms          src/custom_env.py:617-2034  -> gen_2/3/4_rooms()
//   _generate_full_map             src/custom_env.py:332-369   -> gen_single()
//   _generate_{gto,gtg,open,pkp}   src/custom_env.py:371-513   -> gen_single()
//   _generate_{drop,move}_map      src/custom_env.py:515-593   -> gen_single()
//   obstacles (cfg.obstacles)      src/custom_env.py:154-172   -> place_obstacles()
//   'drop' / 'move' missions       src/custom_env.py:214-256   -> gen_attempt(), move_range()
//   next2door                      src/custom_env.py:2036-2046 -> next2door()
//   TokenizeVocabWrapper           src/environment.py:91-112   -> host mission table
//   Discrete2BoxWrapper            src/environment.py:144-149  -> one-hot direction stack
// plus minigrid's MiniGridEnv.step/gen_obs/place_obj/place_agent and Grid.process_vis
// (see_through_walls=False -> apply_vis()) (3P),
// CPython random (_randbelow via getrandbits) and numpy PCG64/Generator.integers (A.6).
#pragma once
#ifndef MGX_HOST_SIM
#include <hip/hip_runtime.h>
#else
// tests/host_gen: the generator compiled for the host (one lane at a time) as a CPU check of its draw
// order against the C oracle; the harness defines the few device intrinsics used here
#include "host_sim.h"
#endif
#include <stdint.h>

#include "mgx_diag.h"

namespace mgx {

// ---------------------------------------------------------------- cell code
// bits 0-3: OBJECT_TO_IDX type (1 empty, 2 wall, 4 door closed/locked, 5 key,
// 6 ball, 7 box, 8 goal, 9 lava, 11 = OPEN door); bits 4-6: COLOR_TO_IDX;
// bit 7: aux (door: locked; box: holds a Key of its colour).  0 = "nothing"
// (only used for the carried-object slot).
constexpr uint8_t CODE_EMPTY = 0x01;
constexpr uint8_t CODE_WALL = 2 | (5 << 4);   // Wall() is grey
constexpr uint8_t CODE_GOAL = 8 | (1 << 4);   // Goal() is green
constexpr uint8_t CODE_LAVA = 9;              // Lava() is red (COLOR_TO_IDX 0)
constexpr int T_EMPTY = 1, T_WALL = 2, T_DOOR = 4, T_KEY = 5, T_BALL = 6, T_BOX = 7,
              T_GOAL = 8, T_LAVA = 9, T_OPEN = 11;
constexpr int A_LEFT = 0, A_RIGHT = 1, A_FORWARD = 2, A_PICKUP = 3, A_DROP = 4,
              A_TOGGLE = 5, A_DONE = 6;
constexpr uint8_t NONE8 = 0xFF;

// COLOR_NAMES (sorted) index -> COLOR_TO_IDX
__device__ __forceinline__ int cn2idx(int cn) { return (0x403512 >> (cn * 4)) & 0xF; }  // {2,1,5,3,0,4}

__device__ __forceinline__ uint8_t mk_code(int t, int cidx, int aux) {
    return (uint8_t)(t | (cidx << 4) | (aux << 7));
}
__device__ __forceinline__ bool is_door(uint8_t c) { int t = c & 15; return t == T_DOOR || t == T_OPEN; }
__device__ __forceinline__ bool can_overlap(uint8_t c) {
    int t = c & 15; return t == T_EMPTY || t == T_GOAL || t == T_LAVA || t == T_OPEN;
}
__device__ __forceinline__ bool can_pickup(uint8_t c) { int t = c & 15; return t >= T_KEY && t <= T_BOX; }

// WorldObj.encode(): returns type | colour<<8 | state<<16
__device__ __forceinline__ uint32_t encode3(uint8_t code) {
    uint32_t t = code & 15, c = (code >> 4) & 7, a = code >> 7;
    uint32_t s = (t == T_DOOR) ? 1u + a : 0u;
    t = (t == T_OPEN) ? (uint32_t)T_DOOR : t;
    return t | (c << 8) | (s << 16);
}

// ------------------------------------------------------------ env state
struct __align__(16) EnvState {
    uint8_t ax, ay, dir, carry;      // carry: cell code, 0 = None
    uint16_t step_count;
    int16_t reward_step;             // step_count at mission completion (self.reward), -1 = None
    uint8_t tx, ty;                  // target_pos, NONE8 = None
    uint8_t target_action;           // NONE8 = None
    uint8_t mission_id;              // cmd | colour-name<<2 | type-slot<<5 (host table)
    uint8_t mission_done;
    uint8_t frames;                  // frames of the current episode in the stack (<= n_stack)
    uint8_t flags;
    uint8_t pad;
};
static_assert(sizeof(EnvState) == 16, "EnvState must be 16 bytes");

// mission ids: cmd | colour-name<<2 | type-slot<<5 for 'go to' / 'toggle' / 'pick up',
// 3 = 'go to goal', MID_DROP = 'drop', MID_MOVE + d = 'move left/right/up/down'
constexpr int CMD_GOTO = 0, CMD_TOGGLE = 1, CMD_PICKUP = 2, CMD_GOTOGOAL = 3;
constexpr int MID_DROP = 128, MID_MOVE = 129;
constexpr int TS_DOOR = 0, TS_KEY = 1, TS_BALL = 2, TS_BOX = 3;
__device__ __forceinline__ int type_slot(int t) {
    return t == T_DOOR ? TS_DOOR : t == T_KEY ? TS_KEY : t == T_BALL ? TS_BALL : TS_BOX;
}

__device__ __forceinline__ double reward_at(int sc, int max_steps) {
    // MiniGridEnv._reward: 1 - 0.9 * (step_count / max_steps), fp64, no contraction
    double q = (double)sc / (double)max_steps;
    double m = __dmul_rn(0.9, q);
    return __dsub_rn(1.0, m);
}

// ------------------------------------------------------------ render
// gen_obs(): 7x7 egocentric view, [c][vx][vy] frame (VecTransposeImage layout).
// View cell (vx,vy) = world A + (6-vy)*dir_vec + (vx-3)*right_vec (== minigrid's
// slice + (dir+1) x rotate_left); out of bounds -> Wall; (3,6) -> carried or None.
template <typename Store>
__device__ __forceinline__ void render_view(const uint8_t *g, int S, int ax, int ay, int dir,
                                            uint8_t carry, Store store) {
    const int dx = (dir == 0) - (dir == 2);
    const int dy = (dir == 1) - (dir == 3);
    const int rx = -dy, ry = dx;
#pragma unroll
    for (int vx = 0; vx < 7; ++vx) {
#pragma unroll
        for (int vy = 0; vy < 7; ++vy) {
            uint8_t code;
            if (vx == 3 && vy == 6) {
                code = carry ? carry : CODE_EMPTY;
            } else {
                int wx = ax + (6 - vy) * dx + (vx - 3) * rx;
                int wy = ay + (6 - vy) * dy + (vx - 3) * ry;
                bool in = (unsigned)wx < (unsigned)S && (unsigned)wy < (unsigned)S;
                code = in ? g[wy * S + wx] : CODE_WALL;
            }
            uint32_t e = encode3(code);
            store(vx * 7 + vy, e);
        }
    }
}

// ------------------------------------------------------------ PCG64 / SeedSequence
constexpr uint64_t PCG_MH = 2549297995355413924ULL, PCG_ML = 4865540595714422341ULL;

struct Pcg {
    uint64_t sh, sl, ih, il;
    uint32_t has, uinteger;
};

__device__ __forceinline__ void pcg_step(Pcg &p) {
    uint64_t lo = p.sl * PCG_ML;
    uint64_t hi = __umul64hi(p.sl, PCG_ML) + p.sl * PCG_MH + p.sh * PCG_ML;
    uint64_t nlo = lo + p.il;
    hi += p.ih + (nlo < lo ? 1ull : 0ull);
    p.sh = hi;
    p.sl = nlo;
}
__device__ __forceinline__ uint64_t pcg_next64(Pcg &p) {
    pcg_step(p);
    uint32_t rot = (uint32_t)(p.sh >> 58);
    uint64_t x = p.sh ^ p.sl;
    return (x >> rot) | (x << ((64u - rot) & 63u));
}
__device__ __forceinline__ uint32_t pcg_next32(Pcg &p) {
    if (p.has) { p.has = 0; return p.uinteger; }
    uint64_t n = pcg_next64(p);
    p.has = 1;
    p.uinteger = (uint32_t)(n >> 32);
    return (uint32_t)n;
}
// Generator.integers(lo, hi) (exclusive hi), scalar path: buffered Lemire32.
__device__ __forceinline__ int pcg_integers(Pcg &p, int lo, int hi) {
    uint32_t rng = (uint32_t)(hi - 1 - lo);
    if (rng == 0) return lo;
    uint32_t rng_excl = rng + 1u;
    // a power-of-two range (every goal / agent / direction draw: integers(0, S) with S = 8 or 16,
    // integers(0, 4)): m = x << k, so the low word is never below the threshold (0) and the draw is
    // x's top k bits -- the same value without the 32 x 32 multiply
    if (rng_excl != 0u && (rng_excl & rng) == 0u) return lo + (int)(pcg_next32(p) >> (32 - __builtin_ctz(rng_excl)));
    uint64_t m = (uint64_t)pcg_next32(p) * rng_excl;
    uint32_t left = (uint32_t)m;
    if (left < rng_excl) {
        uint32_t thr = (0xffffffffu - rng) % rng_excl;
        while (left < thr) {
            m = (uint64_t)pcg_next32(p) * rng_excl;
            left = (uint32_t)m;
        }
    }
    return lo + (int)(m >> 32);
}

// Two consecutive Generator.integers(0, S) draws (a position (x, y), S >= 2) with one PCG64 step and no
// branch on the half-word buffer: the pair always consumes exactly one 64-bit output -- buffered low half
// + the new output's low half (has = 1: the new high half is buffered), or the new output's two halves
// (has = 0; the high half stays in `uinteger`, as the second next32 leaves it) -- so `has` is the same after
// the pair as before.  A Lemire rejection (probability S / 2^32 per
// draw) replays the pair through pcg_integers from the saved state.  Same values and state as two
// pcg_integers(p, 0, S) calls.
__device__ __forceinline__ void pcg_cell(Pcg &p, int S, int &x, int &y) {
    const Pcg p0 = p;
    const uint64_t n = pcg_next64(p);
    const uint32_t lo = (uint32_t)n, hi = (uint32_t)(n >> 32);
    const uint32_t a = p.has ? p.uinteger : lo, b = p.has ? lo : hi;
    p.uinteger = hi;                  // has = 1: the new buffer; has = 0: the (dead) copy next32 leaves behind
    const uint32_t s = (uint32_t)S;
    if ((s & (s - 1u)) == 0u) {                                   // power of two (S = 8, 16): top bits
        const int k = 32 - __builtin_ctz(s);
        x = (int)(a >> k);
        y = (int)(b >> k);
        return;
    }
    const uint64_t ma = (uint64_t)a * s, mb = (uint64_t)b * s;
    if ((uint32_t)ma < s || (uint32_t)mb < s) {                  // Lemire's rejection test may apply: replay
        p = p0;
        x = pcg_integers(p, 0, S);
        y = pcg_integers(p, 0, S);
        return;
    }
    x = (int)(ma >> 32);
    y = (int)(mb >> 32);
}

// numpy SeedSequence(seed).generate_state(4, uint64) -> PCG64 seeding.
__device__ __forceinline__ uint32_t ss_hashmix(uint32_t v, uint32_t &hc) {
    v ^= hc; hc *= 0x931e8875u; v *= hc; v ^= v >> 16; return v;
}
__device__ __forceinline__ uint32_t ss_mix(uint32_t x, uint32_t y) {
    uint32_t r = 0xca01f9ddu * x - 0x4973f715u * y; r ^= r >> 16; return r;
}
__device__ __forceinline__ void pcg_seed(Pcg &p, uint64_t seed) {
    uint32_t e0 = (uint32_t)seed, e1 = (uint32_t)(seed >> 32);
    int nent = (seed >> 32) ? 2 : 1;
    uint32_t pool[4];
    uint32_t hc = 0x43b0d7e5u;
#pragma unroll
    for (int i = 0; i < 4; i++) pool[i] = ss_hashmix(i == 0 ? e0 : (i == 1 && nent == 2 ? e1 : 0u), hc);
#pragma unroll
    for (int s = 0; s < 4; s++)
#pragma unroll
        for (int d = 0; d < 4; d++)
            if (s != d) pool[d] = ss_mix(pool[d], ss_hashmix(pool[s], hc));
    uint32_t w[8];
    uint32_t hb = 0x8b51f9ddu;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint32_t v = pool[i & 3];
        v ^= hb; hb *= 0x58f38dedu; v *= hb; v ^= v >> 16;
        w[i] = v;
    }
    uint64_t v0 = (uint64_t)w[0] | ((uint64_t)w[1] << 32), v1 = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
    uint64_t v2 = (uint64_t)w[4] | ((uint64_t)w[5] << 32), v3 = (uint64_t)w[6] | ((uint64_t)w[7] << 32);
    // initstate = v0:v1, initseq = v2:v3; inc = initseq<<1 | 1
    p.ih = (v2 << 1) | (v3 >> 63);
    p.il = (v3 << 1) | 1ull;
    p.sh = 0; p.sl = 0;
    pcg_step(p);
    uint64_t nl = p.sl + v1;
    p.sh = p.sh + v0 + (nl < p.sl ? 1ull : 0ull);
    p.sl = nl;
    pcg_step(p);
    p.has = 0; p.uinteger = 0;
}

// ------------------------------------------------------------ generator context
// Generation is one long serial RNG chain per env, so its cost is latency: the
// generator therefore keeps everything it tests in registers -- occupancy and
// door-adjacency as S*S-bit masks (NW 64-bit words), the next four MT19937
// words in a register queue -- and only WRITES the cell codes to the LDS grid
// row (read back once, when the finished grid is copied out).
// MT19937 words are consumed ONLY through random._randbelow(n) with n < 32, which
// reads just the top k = bit_length(n) <= 5 bits of each word.  The engine therefore
// keeps the shared MT(seed) output stream as 5-bit fields, ten per u64 group (6-bit
// slots, bit 5 of every slot a zero guard): 5x denser than the words, and a SWAR
// compare tests ten candidate words at once (see randbelow).
constexpr int MT_FIELDS = 10;       // words per packed group
// Groups per lane-private LDS window: 8 (80 words, about one episode's draws) for S <= 8, where the
// refill wave's LDS (13 KB) then fits four to a CU beside four rollout workgroups; 16 for larger grids
// (their LDS budget is set by the grids; the window reloads half as often).
template <int NW>
__host__ __device__ constexpr int mt_wg() { return NW == 1 ? MGX_MT_WG1 : 16; }
constexpr int MT_WG_MAX = 16;
template <int NW>   // dwords per lane window row: 8-B aligned, 2-way banked for b64
__host__ __device__ constexpr int win_stride() { return 2 * mt_wg<NW>() + 2; }
__host__ __device__ constexpr int win_stride_of(int nw) { return nw == 1 ? win_stride<1>() : win_stride<2>(); }
constexpr uint64_t MT_REP = 0x041041041041041ull;   // 1 in every 6-bit slot of ten
constexpr uint64_t MT_LOW60 = (1ull << 60) - 1ull;
constexpr int MAX_OBJS = 32;     // objs list capacity bound; the list is sized per config (KParams.obj_cap)
constexpr int SAT_PROBE = 64;     // rejections before the exhaustive satisfiability probe
constexpr uint32_t PCG_LOOP_LIMIT = 1u << 20;

template <int NW>
struct Bits {                     // S*S-bit set, bit b = y*S + x; named words (no array: stays in VGPRs)
    uint64_t w0, w1, w2, w3;
    __device__ __forceinline__ void clear() { w0 = w1 = w2 = w3 = 0; }
    __device__ __forceinline__ bool test(int b) const {
        const int i = b >> 6;
        uint64_t v = w0;
        if (NW > 1) v = i == 1 ? w1 : v;
        if (NW > 2) { v = i == 2 ? w2 : v; v = i == 3 ? w3 : v; }
        return (v >> (b & 63)) & 1ull;
    }
    __device__ __forceinline__ void set(int b) {
        const int i = b >> 6;
        const uint64_t m = 1ull << (b & 63);
        w0 |= i == 0 ? m : 0ull;
        if (NW > 1) w1 |= i == 1 ? m : 0ull;
        if (NW > 2) { w2 |= i == 2 ? m : 0ull; w3 |= i == 3 ? m : 0ull; }
    }
    __device__ __forceinline__ void unset(int b) {
        const int i = b >> 6;
        const uint64_t m = ~(1ull << (b & 63));
        w0 &= i == 0 ? m : ~0ull;
        if (NW > 1) w1 &= i == 1 ? m : ~0ull;
        if (NW > 2) { w2 &= i == 2 ? m : ~0ull; w3 &= i == 3 ? m : ~0ull; }
    }
};

// S > 11 (four 64-bit words): a register mask set makes the generator state too
// large to stay in VGPRs; there the generator reads its LDS grid row instead.
template <>
struct Bits<4> {
    __device__ __forceinline__ void clear() {}
    __device__ __forceinline__ void set(int) {}
    __device__ __forceinline__ void unset(int) {}
};

template <int NW>
struct Gen {
    uint8_t *g;            // LDS grid row (S*S used, row-major y*S+x), write-mostly
    int S;
    Bits<NW> occ;          // cell holds an object (walls, doors, goal, keys, boxes, balls)
    Bits<NW> dn;           // cell is next to a door (custom_env.py:2036-2046)
    // MT19937 shared table + cursor: q0..q3 = table[cur .. cur+3]
    const uint64_t *table; // packed MT19937 field groups (global ring of rmask+1 groups + mirror pad)
    uint64_t rmask;        // ring slots - 1 (a power of two): group g lives in slot g & rmask
    uint64_t tlo, thi;     // groups [tlo, thi) of the stream are in the ring (mgx_mt_slide_kernel)
    uint64_t *win;         // LDS window: packed groups [gbase, gbase + mt_wg<NW>())
    uint64_t gbase;        // first group in the window
    uint64_t cur, astart;  // word cursor; first word of the current reset attempt
    uint64_t ga, gb, gc;   // packed groups g, g+1 (ready), g+2 (LDS read in flight), g = cur / 10
    uint64_t gi;           // g (kept with the queue: no 64-bit division per group rotation)
    int go;                // cur % 10
    uint32_t llw;
    bool abort;
    uint32_t err;
    Pcg pcg;
    int ax, ay, adir;
    int goalx, goaly;      // the first Goal added to objs (-1: none): the 'go to goal' target without a scan
    bool phave;            // gen_multi: this attempt's MT-only prefix comes from prec (a record looked up by the refill)
    uint64_t prec;
    uint32_t *objs;        // LDS objs list: type | cname<<4 | x<<8 | y<<16 (cname 15 = None)
    int nobjs;
    uint32_t tmask;        // bit t: an object of type t is in objs
    // config
    int problem, cfg_mission, num_objects, all_doors_open, n_obstacles;
#if MGX_GEN_STAMPS
    unsigned long long *stamps;   // diagnostic build: per-section wave clocks (counters[8..])
    uint64_t tlast;
#endif
};

// Diagnostic section clock (MGX_GEN_STAMPS builds only): the first active lane of
// the wave adds the shader clocks since this lane's previous stamp to counter k.
#if MGX_GEN_STAMPS
#define GSTAMP(G, k)                                                                     \
    do {                                                                                 \
        const uint64_t _t = __builtin_amdgcn_s_memtime();                                \
        const unsigned long long _m = __ballot(1);                                       \
        if ((int)__lane_id() == __ffsll((long long)_m) - 1) atomicAdd(&(G).stamps[k], _t - (G).tlast); \
        (G).tlast = _t;                                                                  \
    } while (0)
#if MGX_GEN_STAMPS == 2          // section clocks only (no per-iteration counters: less distortion)
#define GCOUNT(G, k) do { } while (0)
#else
#define GCOUNT(G, k)                                                                     \
    do {                                                                                 \
        const unsigned long long _m = __ballot(1);                                       \
        if ((int)__lane_id() == __ffsll((long long)_m) - 1) atomicAdd(&(G).stamps[k], 1ull); \
    } while (0)
#endif
#else
#define GSTAMP(G, k) do { } while (0)
#define GCOUNT(G, k) do { } while (0)
#endif

// MGX_GEN_SKIP (mgx_diag.h): elimination builds that skip generator sections.

template <int NW>
__device__ __forceinline__ void put(Gen<NW> &G, int x, int y, uint8_t code) {   // grid.set(x, y, obj)
    const int b = y * G.S + x;
    G.g[b] = code;
    if (code == CODE_EMPTY) G.occ.unset(b); else G.occ.set(b);
}

// Refill the lane's LDS window with packed groups [g, g + MT_WG) from ring slot g & rmask (the
// ring is followed by a mirror of its first MT_PAD slots, so the 16 groups are contiguous): 16
// independent 16-B global loads in flight (one L2/HBM round trip), 32 b64 LDS stores.
// Out of line: it is the cold path of every draw site (inlined at each of them it
// made the generator ~2k instructions larger).
#ifndef MGX_HOST_SIM
typedef __attribute__((address_space(3))) uint64_t lds_u64;
#else
typedef uint64_t lds_u64;
#endif
constexpr int MT_PAD = MT_WG_MAX + 4;   // mirror pad groups after the ring (a window may start in its last slot)
template <int WG>
__device__ __noinline__ void mt_refill_cold(const uint64_t *__restrict__ table, uint64_t slot, lds_u64 *win) {
    const uint4 *src = reinterpret_cast<const uint4 *>(table + slot);
    static_assert(WG % 8 == 0 && WG <= MT_WG_MAX, "window loads go in fours of 16 B");
#pragma unroll
    for (int h = 0; h < WG / 8; h++) {            // (4 loads in flight, then 8 LDS stores) per 8 groups
        const uint4 v0 = src[4 * h], v1 = src[4 * h + 1], v2 = src[4 * h + 2], v3 = src[4 * h + 3];
        lds_u64 *d = win + 8 * h;
        d[0] = (uint64_t)v0.x | ((uint64_t)v0.y << 32); d[1] = (uint64_t)v0.z | ((uint64_t)v0.w << 32);
        d[2] = (uint64_t)v1.x | ((uint64_t)v1.y << 32); d[3] = (uint64_t)v1.z | ((uint64_t)v1.w << 32);
        d[4] = (uint64_t)v2.x | ((uint64_t)v2.y << 32); d[5] = (uint64_t)v2.z | ((uint64_t)v2.w << 32);
        d[6] = (uint64_t)v3.x | ((uint64_t)v3.y << 32); d[7] = (uint64_t)v3.z | ((uint64_t)v3.w << 32);
    }
}
template <int NW>
__device__ __forceinline__ uint64_t win_group(Gen<NW> &G, uint64_t g) {
    constexpr int MT_WG = mt_wg<NW>();
    uint64_t off = g - G.gbase;
    if (off >= MT_WG) {
        GCOUNT(G, 23);
        // groups outside [tlo, thi) are not (or no longer) in the ring: MGX_DEVERR_MT_TABLE
        if (g < G.tlo || g + MT_WG > G.thi) G.err |= 1u;
        mt_refill_cold<MT_WG>(G.table, g & G.rmask, (lds_u64 *)G.win);
        G.gbase = g;
        off = 0;
    }
    return G.win[off];
}
__device__ __forceinline__ uint64_t div10(uint64_t v) { return __umul64hi(v, 0xCCCCCCCCCCCCCCCDull) >> 3; }
// (re)load the group registers at the current cursor
template <int NW>
__device__ __forceinline__ void mt_sync(Gen<NW> &G) {
    const uint64_t g = div10(G.cur);
    G.go = (int)(G.cur - g * MT_FIELDS);
    G.gi = g;
    G.ga = win_group(G, g);
    G.gb = win_group(G, g + 1);
    G.gc = win_group(G, g + 2);
}
// random._randbelow_with_getrandbits(n), 1 <= n < 32 (live-lock capped).
// The reference draws getrandbits(k) = word >> (32 - k) until it is < n; on the 5-bit
// field f of a word that is f < n << (5 - k).  Ten fields at once: guard-bit SWAR
// subtract, first set guard = first accepted word.  One pass almost always suffices
// (a lane needs another only after ten rejections), so lanes do not diverge here.
struct RbConst {            // randbelow(n) constants: field shift 5 - bit_length(n), SWAR compare word
    uint64_t c1;
    uint32_t sh;
};
__device__ __forceinline__ RbConst rb_const(uint32_t n) {
    const uint32_t sh = 5u - (uint32_t)(32 - __clz(n));
    return RbConst{(uint64_t)(32u + (n << sh) - 1u) * MT_REP, sh};   // per slot: 32 + c - 1
}
template <int NW>
__device__ __forceinline__ int randbelow_c(Gen<NW> &G, const RbConst K);
template <int NW>
__device__ __forceinline__ int randbelow(Gen<NW> &G, uint32_t n) {
    GCOUNT(G, 24);
    if (n >= 32u) { G.err |= 8u; return 0; }        // excluded by validation (n < 32 always)
    return randbelow_c(G, rb_const(n));
}
template <int NW>
__device__ __forceinline__ int randbelow_c(Gen<NW> &G, const RbConst K) {
    const uint64_t c1 = K.c1;
    const uint32_t sh = K.sh;
    for (;;) {
        GCOUNT(G, 21);
        const int o6 = (int)__umul24((uint32_t)G.go, 6u);
        const uint64_t f = ((G.ga >> o6) | (G.gb << (60 - o6))) & MT_LOW60;  // words cur..cur+9
        const uint64_t acc = (c1 - f) & (32ull * MT_REP);   // guard bit of slot i <=> field i < c
        const uint32_t left = G.llw - (uint32_t)(G.cur - G.astart);   // words this attempt may still take
        const int j = acc ? (int)(((uint32_t)__ffsll((long long)acc) - 1u - 5u) * 171u >> 10) : MT_FIELDS;
        int m = j < MT_FIELDS ? j + 1 : MT_FIELDS;         // words consumed by this pass
        if ((uint32_t)m > left) {                           // cap reached before an accepted word
            G.cur = G.astart + G.llw;
            G.abort = true;
            return 0;
        }
        const int r = (int)(((f >> (6 * (j < MT_FIELDS ? j : 0))) & 31u) >> sh);
        G.cur += (uint64_t)m;
        G.go += m;
        if (G.go >= MT_FIELDS) {                            // next group: rotate, prefetch two ahead
            G.go -= MT_FIELDS;
            G.ga = G.gb;
            G.gb = G.gc;
            G.gi++;
            G.gc = win_group(G, G.gi + 2);
        }
        if (j < MT_FIELDS) return r;
    }
}
// consume m <= 10 words of the register queue
template <class GT>
__device__ __forceinline__ void mt_advance(GT &G, int m) {
    G.cur += (uint64_t)m;
    G.go += m;
    if (G.go >= MT_FIELDS) {
        G.go -= MT_FIELDS;
        G.ga = G.gb;
        G.gb = G.gc;
        G.gi++;
        G.gc = win_group(G, G.gi + 2);
    }
}
// `cnt` (<= 12) successive _randbelow draws whose moduli are known up front -- draw i's modulus in bits
// 5i..5i+4 of `prog`, its value returned in the same bits: the door draws of the room generators (colour,
// locked, key-in-box per door, then the door positions, custom_env.py:635-650, 878-930, 1322-1391) and the
// mission / room-count draws before them.  Each pass over the ten words of the register queue decodes as
// many consecutive draws as it holds (draw i = the first word after draw i-1's that passes draw i's test,
// one SWAR compare and a find-first-set each); a draw that finds no accepted word in the rest of the ten
// consumes them all and continues in the next pass.  Word consumption and the live-lock cap are those of
// cnt randbelow() calls, which spent a whole pass (and its group rotation) per draw (round 4).
template <class GT>
__device__ __forceinline__ uint64_t randbelow_seq(GT &G, uint64_t prog, int cnt) {
    constexpr uint64_t GM = 32ull * MT_REP;              // guard bit of every slot
    uint64_t res = 0;
    int i = 0;
#pragma unroll 1
    while (i < cnt) {
        GCOUNT(G, 21);
        const int o6 = (int)__umul24((uint32_t)G.go, 6u);
        const uint64_t f = ((G.ga >> o6) | (G.gb << (60 - o6))) & MT_LOW60;   // words cur..cur+9
        uint64_t avail = GM;                             // slots after the last decoded draw
        int used = MT_FIELDS;                            // words this pass consumes
#pragma unroll 1
        while (i < cnt) {
            const RbConst K = rb_const((uint32_t)(prog >> (5 * i)) & 31u);
            const uint64_t acc = (K.c1 - f) & avail;
            if (!acc) { used = MT_FIELDS; break; }       // draw i runs past these ten words
            const int b = __ffsll((long long)acc) - 1;   // guard bit 6 j + 5 of the accepted word j
            res |= (uint64_t)((((uint32_t)(f >> (b - 5))) & 31u) >> K.sh) << (5 * i);
            avail &= ~((2ull << b) - 1ull);
            used = (int)((uint32_t)(b + 1) * 171u >> 10);   // j + 1
            i++;
        }
        const uint32_t left = G.llw - (uint32_t)(G.cur - G.astart);
        if ((uint32_t)used > left) {                     // the cap comes before the sequence's end
            G.cur = G.astart + G.llw;
            G.abort = true;
            return res;
        }
        mt_advance(G, used);
    }
    return res;
}
// The reference's rejection loop `while True: x = randint(x0, x1); y = randint(y0, y1);
// if ok(x, y): break` (two _randbelow per draw) with the rejected cells as a bit set.  One SWAR
// pass over the next ten words finds every complete draw they hold: x is the first word passing
// x's test, y the first after it passing y's, the next x the first after that...  so a rejected
// draw costs a few bit operations instead of two randbelow calls.  A draw that straddles the
// ten words is taken word by word (randbelow_c).  Word consumption and the live-lock cap are
// exactly randbelow's: the attempt is abandoned when a draw would need a word past the cap.
// has_c: the draw is preceded by one more _randbelow (modulus KC: an object placement's
// random.choice(obj_choice), custom_env.py:662-667 -- no MT word is drawn between the two), decoded from
// the first pass's words before the cell candidates (round 4: it took a randbelow pass of its own) ->
// `choice`.
template <int NW, typename Bad, typename Sat>
__device__ __forceinline__ void draw_cell(Gen<NW> &G, const RbConst KX, const RbConst KY, int x0, int y0, int &x, int &y,
                                          Bad bad, Sat sat /* probe after SAT_PROBE rejections; null: none */,
                                          bool has_c, const RbConst KC, int &choice) {
    constexpr uint64_t GM = 32ull * MT_REP;              // guard bit of every slot
    int rej = 0;
    bool need_c = has_c;
#pragma unroll 1
    for (;;) {
        GCOUNT(G, 21);
        const int o6 = (int)__umul24((uint32_t)G.go, 6u);
        const uint64_t f = ((G.ga >> o6) | (G.gb << (60 - o6))) & MT_LOW60;   // words cur..cur+9
        uint64_t avail = GM;                             // slots not consumed by an earlier draw
        int used = 0;                                    // words through the last draw examined
        if (need_c) {
            const uint64_t acc = (KC.c1 - f) & GM;
            if (!acc) {                                  // the choice runs past these ten words
                const uint32_t left = G.llw - (uint32_t)(G.cur - G.astart);
                if ((uint32_t)MT_FIELDS > left) {
                    G.cur = G.astart + G.llw;
                    G.abort = true;
                    return;
                }
                mt_advance(G, MT_FIELDS);
                continue;
            }
            const int b = __ffsll((long long)acc) - 1;
            choice = (int)((((uint32_t)(f >> (b - 5))) & 31u) >> KC.sh);
            avail &= ~((2ull << b) - 1ull);
            used = (int)((uint32_t)(b + 1) * 171u >> 10);
            need_c = false;
        }
        const uint64_t accx = (KX.c1 - f) & GM, accy = (KY.c1 - f) & GM;    // slot passes x's / y's test
        bool ok = false;
#pragma unroll 1
        for (;;) {
            const uint64_t cx = accx & avail;
            if (!cx) break;
            const int bx = __ffsll((long long)cx) - 1;                   // guard bit 6 jx + 5
            const uint64_t cy = accy & avail & ~((2ull << bx) - 1ull);
            if (!cy) break;
            const int by = __ffsll((long long)cy) - 1;
            x = x0 + (int)(((uint32_t)(f >> (bx - 5)) & 31u) >> KX.sh);
            y = y0 + (int)(((uint32_t)(f >> (by - 5)) & 31u) >> KY.sh);
            used = (int)((uint32_t)(by + 1) * 171u >> 10);               // jy + 1
            avail &= ~((2ull << by) - 1ull);
            if (!bad(x, y)) { ok = true; break; }
            if (++rej == SAT_PROBE && !sat()) { live_lock(G); return; }
        }
        const uint32_t left = G.llw - (uint32_t)(G.cur - G.astart);
        if ((uint32_t)used > left) {                     // a draw would pass the cap
            G.cur = G.astart + G.llw;
            G.abort = true;
            return;
        }
        mt_advance(G, used);
        if (ok) return;
        x = x0 + randbelow_c(G, KX);                     // the draw across the window's end
        y = y0 + randbelow_c(G, KY);
        if (G.abort) return;
        if (!bad(x, y)) return;
        if (++rej == SAT_PROBE && !sat()) { live_lock(G); return; }
    }
}

template <int NW>
__device__ __forceinline__ int randint(Gen<NW> &G, int a, int b) { return a + randbelow(G, (uint32_t)(b - a + 1)); }
template <int NW>
__device__ __forceinline__ bool choice_bool(Gen<NW> &G) { return randbelow(G, 2) == 0; }   // choice([True, False])

template <int NW>
__device__ __forceinline__ bool next2door(const Gen<NW> &G, int x, int y) {
    if constexpr (NW == 4) {
        return is_door(G.g[y * G.S + x - 1]) || is_door(G.g[y * G.S + x + 1]) ||
               is_door(G.g[(y - 1) * G.S + x]) || is_door(G.g[(y + 1) * G.S + x]);
    } else {
        return G.dn.test(y * G.S + x);
    }
}
template <int NW>
__device__ __forceinline__ bool occupied(const Gen<NW> &G, int b) {
    if constexpr (NW == 4) return G.g[b] != CODE_EMPTY;
    else return G.occ.test(b);
}

// objs entry: type | cname<<4 | x<<8 | y<<16 | OBJ_KEYFLAG (a door's key / key box, placed by the
// key task: tells the scene description's key lines from object lines, mgx_scene)
constexpr uint32_t OBJ_KEYFLAG = 1u << 24;
template <int NW>
__device__ __forceinline__ void add_obj(Gen<NW> &G, int t, int cname, int x, int y, uint32_t flags = 0) {
    // branchless flags: with `if (full) { err |= 8; return; } ... tmask |= bit` the compiler sinks the
    // two ORs into one through a select of &err / &tmask, which puts both fields on the stack
    // (scratch loads with a full vmcnt wait in every placement)
    const bool full = G.nobjs >= MAX_OBJS;
    G.err |= full ? 8u : 0u;
    G.tmask |= full ? 0u : 1u << t;
    const bool first_goal = !full && t == T_GOAL && G.goalx < 0;
    G.goalx = first_goal ? x : G.goalx;
    G.goaly = first_goal ? y : G.goaly;
    if (!full)
        G.objs[G.nobjs++] = (uint32_t)t | ((uint32_t)(cname & 15) << 4) | ((uint32_t)x << 8) | ((uint32_t)y << 16) | flags;
}

// MiniGridEnv.place_obj position draw over the whole grid (PCG64): rejects occupied
// cells and the agent's cell; `commit` decides what (if anything) lands there.
template <int NW>
__device__ __forceinline__ void draw_free_cell(Gen<NW> &G, int &px, int &py) {
    for (uint32_t it = 0;; ++it) {
        GCOUNT(G, 22);
        if (it > PCG_LOOP_LIMIT) { G.err |= 4u; px = 1; py = 1; return; }
        int x, y;
        pcg_cell(G.pcg, G.S, x, y);
        if (occupied(G, y * G.S + x)) continue;
        if (x == G.ax && y == G.ay) continue;
        px = x; py = y;
        return;
    }
}
template <int NW>
__device__ __forceinline__ void place_agent(Gen<NW> &G) {        // place_obj(None) + random dir
    G.ax = -1; G.ay = -1;
    int x, y;
    draw_free_cell(G, x, y);
    G.ax = x; G.ay = y;
    G.adir = pcg_integers(G.pcg, 0, 4);
}

// ---- ordered choice lists as bitmasks (list.remove keeps order) --------------
// element b of an obj_choice list = (types[b / 6], COLOR_NAMES[b % 6])
__device__ __forceinline__ int nth_set_bit(uint32_t m, int r) {   // branchless rank-select, r < popc(m)
    int pos = 0, c;
    c = __popc(m & 0xFFFFu); if (r >= c) { r -= c; m >>= 16; pos += 16; }
    c = __popc(m & 0xFFu);   if (r >= c) { r -= c; m >>= 8;  pos += 8; }
    c = __popc(m & 0xFu);    if (r >= c) { r -= c; m >>= 4;  pos += 4; }
    c = __popc(m & 0x3u);    if (r >= c) { r -= c; m >>= 2;  pos += 2; }
    c = (int)(m & 1u);       if (r >= c) { pos += 1; }
    return pos;
}
template <int NW>
__device__ __forceinline__ int mask_choice(Gen<NW> &G, uint32_t m) {   // index into the list
    return nth_set_bit(m, randbelow(G, (uint32_t)__popc(m)));
}

template <int NW>
__device__ __forceinline__ void live_lock(Gen<NW> &G) {
    // provably unsatisfiable `while True` loop: the reference would spin until the
    // cap; that consumes exactly llw words of this attempt -- jump there.
    G.cur = G.astart + G.llw;
    G.abort = true;
}

// `while True: p=(randint(x0,x1), randint(y0,y1)); if p!=goal and [p!=agent] and
//  [p!=other] and not next2door(p): break` -> grid.set(Box(c,Key(c)) | Key(c)); objs.append
template <int NW>
__device__ __forceinline__ void place_key(Gen<NW> &G, int x0, int x1, int y0, int y1, int gx, int gy, bool chk_agent,
                                          int ox, int oy, int cname, bool kib, int *kx, int *ky) {
    int x, y, rej = 0;
    for (;;) {
        x = randint(G, x0, x1);
        y = randint(G, y0, y1);
        if (G.abort) return;
        const bool bad = (x == gx && y == gy) || (chk_agent && x == G.ax && y == G.ay) || (x == ox && y == oy) ||
                         next2door(G, x, y);
        if (!bad) break;
        if (++rej == SAT_PROBE) {
            bool sat = false;
            for (int xx = x0; xx <= x1 && !sat; xx++)
                for (int yy = y0; yy <= y1 && !sat; yy++)
                    sat = !((xx == gx && yy == gy) || (chk_agent && xx == G.ax && yy == G.ay) ||
                            (xx == ox && yy == oy) || next2door(G, xx, yy));
            if (!sat) { live_lock(G); return; }
        }
    }
    const int cidx = cn2idx(cname);
    if (kib) { put(G, x, y, mk_code(T_BOX, cidx, 1)); add_obj(G, T_BOX, cname, x, y, OBJ_KEYFLAG); }
    else { put(G, x, y, mk_code(T_KEY, cidx, 0)); add_obj(G, T_KEY, cname, x, y, OBJ_KEYFLAG); }
    if (kx) { *kx = x; *ky = y; }
}

// `for _ in range(n): (t,c)=choice(obj_choice); obj_choice.remove((t,c)); while True:
//  p=(randint..); [p in objs -> retry]; if p != agent and not next2door(p): break; put_obj`
// (p in objs <=> cell occupied, inside a room interior)
template <int NW>
__device__ __forceinline__ void place_objects(Gen<NW> &G, uint32_t &oc, const int *types, int n, int x0, int x1,
                                              int y0, int y1) {
    for (int k = 0; k < n; k++) {
        if (oc == 0) { G.err |= 8u; return; }
        const int b = mask_choice(G, oc);
        if (G.abort) return;
        oc &= ~(1u << b);
        const int t = types[b / 6], cname = b % 6;
        int x, y, rej = 0;
        for (;;) {
            x = randint(G, x0, x1);
            y = randint(G, y0, y1);
            if (G.abort) return;
            const bool bad = occupied(G, y * G.S + x) || (x == G.ax && y == G.ay) || next2door(G, x, y);
            if (!bad) break;
            if (++rej == SAT_PROBE) {
                bool sat = false;
                for (int xx = x0; xx <= x1 && !sat; xx++)
                    for (int yy = y0; yy <= y1 && !sat; yy++)
                        sat = !(occupied(G, yy * G.S + xx) || (xx == G.ax && yy == G.ay) || next2door(G, xx, yy));
                if (!sat) { live_lock(G); return; }
            }
        }
        put(G, x, y, mk_code(t, cn2idx(cname), 0));
        add_obj(G, t, cname, x, y);
    }
}

__device__ __forceinline__ int door_code(int cname, bool locked, bool open) {
    return open ? mk_code(T_OPEN, cn2idx(cname), 0) : mk_code(T_DOOR, cn2idx(cname), locked ? 1 : 0);
}

template <int NW>
__device__ __forceinline__ void put_door(Gen<NW> &G, int x, int y, uint8_t code) {
    put(G, x, y, code);
    const int S = G.S, b = y * S + x;
    if (x > 0) G.dn.set(b - 1);
    if (x < S - 1) G.dn.set(b + 1);
    if (y > 0) G.dn.set(b - S);
    if (y < S - 1) G.dn.set(b + S);
}

// Cells [x0, x1] x [y0, y1] that a placement loop would accept, as row masks of the
// register bit sets (S <= 11): none -> the reference's `while True` never ends, so the
// live-lock policy applies at once instead of after SAT_PROBE rejected draws (same
// end state: the attempt's cursor jumps to its cap).  Excluded points: (-1,-1) = none.
template <int NW>
__device__ __forceinline__ uint32_t bits_row(const Bits<NW> &B, int y, int S) {
    const int b = y * S;
    uint64_t v = b < 64 ? (B.w0 >> b) : 0ull;
    if (NW > 1) {
        if (b >= 64) v = B.w1 >> (b - 64);
        else if (b + S > 64) v |= B.w1 << (64 - b);
    }
    return (uint32_t)v & ((1u << S) - 1u);
}
template <int NW>
__device__ __forceinline__ bool rect_has_free(const Gen<NW> &G, int x0, int x1, int y0, int y1, bool use_occ,
                                              int ax, int ay, int bx, int by, int cx, int cy) {
    if constexpr (NW == 4) {
        return true;                      // S > 11: the in-loop SAT_PROBE check handles it
    } else {
        const uint32_t rowmask = ((1u << (x1 - x0 + 1)) - 1u) << x0;
        bool sat = false;
        for (int y = y0; y <= y1; y++) {
            uint32_t bad = bits_row(G.dn, y, G.S);
            if (use_occ) bad |= bits_row(G.occ, y, G.S);
            if (ay == y && ax >= 0) bad |= 1u << ax;
            if (by == y && bx >= 0) bad |= 1u << bx;
            if (cy == y && cx >= 0) bad |= 1u << cx;
            sat |= (rowmask & ~bad) != 0;
        }
        return sat;
    }
}

// ---- multi-room layouts, table-driven (custom_env.py:617-2034) ---------------
// One generic pass reproduces _generate_2/3/4_rooms: same RNG draws in the same
// order, same Q1/Q5 quirks, one call site per primitive (keeps the generator
// in registers).  Doors are indexed in the reference's draw order:
//   2 rooms: 0 = vertical door;  3 rooms: 0 = h, 1 = vu, 2 = vl;
//   4 rooms: 0 = hl, 1 = hr, 2 = vu, 3 = vl.
// Rooms are visited in the reference's order:
//   2: L, R;  3: UL, LL, R;  4: UL, LL, UR, LR.

// door d of an nr-room layout: horizontal (x drawn, y = mid) or vertical; range lo..hi
__device__ __forceinline__ void door_geom(int nr, int d, int mid, int S, bool &horiz, int &lo, int &hi) {
    if (nr == 2) { horiz = false; lo = 1; hi = S - 2; return; }
    if (nr == 3) {
        horiz = d == 0;
        lo = d == 2 ? mid + 1 : 1;
        hi = d == 2 ? S - 2 : mid - 1;
        return;
    }
    horiz = d < 2;
    const bool upper_half = (d == 0 || d == 2);
    lo = upper_half ? 1 : mid + 1;
    hi = upper_half ? mid - 1 : S - 2;
}

__device__ __forceinline__ int room_of(int nr, int x, int y, int mid) {
    const bool left = x < mid, up = y < mid;
    if (nr == 2) return left ? 0 : 1;
    if (nr == 3) return left ? (up ? 0 : 1) : 2;
    return left ? (up ? 0 : 1) : (up ? 2 : 3);
}

__device__ __forceinline__ void room_rect(int nr, int r, int mid, int S, int &x0, int &x1, int &y0, int &y1) {
    const bool left = (nr == 2) ? r == 0 : r <= 1;
    const bool full_h = nr == 2 || (nr == 3 && r == 2);
    const bool up = (r == 0) || (nr == 4 && r == 2);
    x0 = left ? 1 : mid + 1; x1 = left ? mid - 1 : S - 2;
    y0 = full_h ? 1 : (up ? 1 : mid + 1); y1 = full_h ? S - 2 : (up ? mid - 1 : S - 2);
}

// keys placed in room r given the agent's room ar: kA, kB door indices (-1 none);
// chk = the agent-room form (agent + other-key checks)
__device__ __forceinline__ void key_spec(int nr, int r, int ar, int &kA, int &kB, bool &chk) {
    kA = -1; kB = -1; chk = (r == ar);
    if (nr == 2) { if (r == ar) kA = 0; return; }
    if (nr == 3) {
        if (r != ar) return;
        if (r == 0) { kA = 1; kB = 0; }        // UL: vu, h
        else if (r == 1) { kA = 2; kB = 0; }   // LL: vl, h
        else { kA = 2; kB = 1; }               // R : vl, vu
        return;
    }
    const int HL = 0, HR = 1, VU = 2, VL = 3;
    if (r == 0) {        // UL
        if (ar == 0) { kA = VU; kB = HL; } else if (ar == 1) kA = VU; else if (ar == 2) kA = HL;
    } else if (r == 1) { // LL
        if (ar == 1) { kA = VL; kB = HL; } else if (ar == 3) kA = HL; else if (ar == 0) kA = VL;
    } else if (r == 2) { // UR
        if (ar == 2) { kA = VU; kB = HR; } else if (ar == 3) kA = VU; else if (ar == 0) kA = HR;
    } else {             // LR
        if (ar == 3) { kA = VL; kB = HR; } else if (ar == 1) kA = HR; else if (ar == 2) kA = VL;
    }
}

__device__ const int MULTI_TYPES[3] = {T_KEY, T_BALL, T_BOX};

// ---- the MT-only prefix of a multi-room attempt (round 6) -----------------------------------------------------
// Everything gen_multi / gen_rooms draw before their first PCG64 draw comes from the shared MT19937 stream only:
// [the mission choice] and randint(2, 4) (custom_env.py:595-615), per door its colour / locked / key_in_box draws
// (:635-643, 878-908, 1322-1362), per door its position [and is_open] (:646-650, 911-930, 1365-1391).  Every env
// reads the same stream (quirk Q7), so the prefix is a pure function of the attempt's first word: the MT slide
// computes it once per stream position (mgx_prefix_kernel, a record per word: KParams.pfx) and the refill looks it
// up instead of drawing (round-6 measurement: running every prefix sequence twice cost the refill 11 us of 155 per
// 20-step epoch at config 2 and 55 of 370 per 64-step epoch at config 4).  One function draws it for both.
struct Prefix {
    int nr, rc;            // rooms; the mission draw (when the config names no mission)
    uint32_t dinfo;        // per door byte: colour | locked << 3 | key_in_box << 4
    uint32_t dpos;         // per door nibble: position - lo (door_geom)
    uint32_t dopen;        // per door bit: is_open (all_doors_open)
};
template <class GT>
__device__ __forceinline__ void prefix_draws(GT &G, int S, bool draw_cmd, bool ado, Prefix &P) {
    const uint64_t r = randbelow_seq(G, draw_cmd ? (4ull | (3ull << 5)) : 3ull, draw_cmd ? 2 : 1);
    P.rc = draw_cmd ? (int)(r & 31) : 0;
    P.nr = 2 + (int)((draw_cmd ? r >> 5 : r) & 31);
    P.dinfo = P.dpos = P.dopen = 0;
    if (G.abort || (MGX_GEN_SKIP & 8)) return;
    const int nr = P.nr, mid = S / 2, ndoors = nr == 2 ? 1 : nr;
    // colour / locked / key_in_box: random.choice(door_colors) of the 6 - d colours left = randbelow(6 - d),
    // locked = choice([True, False]) = randbelow(2) == 0 (not drawn when all_doors_open), key_in_box likewise
    uint64_t prog = 0;
    int cnt = 0;
#pragma unroll 1
    for (int d = 0; d < ndoors; d++) {
        prog |= (uint64_t)(6 - d) << (5 * cnt++);
        if (!ado) prog |= 2ull << (5 * cnt++);
        prog |= 2ull << (5 * cnt++);
    }
    const uint64_t dr = randbelow_seq(G, prog, cnt);
    if (G.abort) return;
    uint32_t dc = 0x3Fu;       // door_colors
#pragma unroll 1
    for (int d = 0, k = 0; d < ndoors; d++) {
        const int col = nth_set_bit(dc, (int)(dr >> (5 * k++)) & 31);
        dc &= ~(1u << col);
        const bool lk = ado ? false : ((dr >> (5 * k++)) & 31) == 0;
        const bool kib = ((dr >> (5 * k++)) & 31) == 0;
        P.dinfo |= (uint32_t)(col | (lk << 3) | (kib << 4)) << (8 * d);
    }
    // door positions: randint(lo, hi) = lo + randbelow(hi - lo + 1) per door [+ is_open], again one sequence
    prog = 0;
    cnt = 0;
#pragma unroll 1
    for (int d = 0; d < ndoors; d++) {
        bool horiz; int lo, hi;
        door_geom(nr, d, mid, S, horiz, lo, hi);
        prog |= (uint64_t)(hi - lo + 1) << (5 * cnt++);
        if (ado) prog |= 2ull << (5 * cnt++);
    }
    const uint64_t pr = randbelow_seq(G, prog, (MGX_GEN_SKIP & 2) ? 0 : cnt);
    if (G.abort) return;
#pragma unroll 1
    for (int d = 0, k = 0; d < ((MGX_GEN_SKIP & 2) ? 0 : ndoors); d++) {
        P.dpos |= (uint32_t)((pr >> (5 * k++)) & 15) << (4 * d);
        if (ado) P.dopen |= (uint32_t)(((pr >> (5 * k++)) & 31) == 0) << d;
    }
}
// A prefix record (u64): [0, 8) words the prefix consumed (1..255; 0 = no record), [8, 16) the wrap count of its
// first word's MT ring slot (stale records of an earlier pass through the ring never match), [16, 18) rooms - 2,
// [18, 20) the mission draw, then per door 10 bits: colour | locked << 3 | key_in_box << 4 | position << 5 | is_open << 9
constexpr int PFX_LOOK = 320;       // words past a position its record may read (255 consumed + a 30-word queue)
__host__ __device__ __forceinline__ uint64_t pfx_pack(const Prefix &P, uint32_t adv, uint32_t tag) {
    uint64_t r = (uint64_t)(adv & 0xFF) | ((uint64_t)(tag & 0xFF) << 8) | ((uint64_t)(P.nr - 2) << 16) |
                 ((uint64_t)(P.rc & 3) << 18);
    for (int d = 0; d < 4; d++)
        r |= (uint64_t)(((P.dinfo >> (8 * d)) & 31) | (((P.dpos >> (4 * d)) & 15) << 5) | (((P.dopen >> d) & 1) << 9))
             << (20 + 10 * d);
    return r;
}
__host__ __device__ __forceinline__ void pfx_unpack(uint64_t r, Prefix &P) {
    P.nr = 2 + (int)((r >> 16) & 3);
    P.rc = (int)((r >> 18) & 3);
    P.dinfo = P.dpos = P.dopen = 0;
    for (int d = 0; d < 4; d++) {
        const uint32_t f = (uint32_t)(r >> (20 + 10 * d)) & 0x3FFu;
        P.dinfo |= (f & 31u) << (8 * d);
        P.dpos |= ((f >> 5) & 15u) << (4 * d);
        P.dopen |= ((f >> 9) & 1u) << d;
    }
}

template <int NW>
__device__ __forceinline__ void gen_rooms(Gen<NW> &G, const Prefix &P) {
    const int S = G.S, mid = S / 2, nr = P.nr;
    if (MGX_GEN_SKIP & 8) { G.ax = 1; G.ay = 1; put(G, S - 2, S - 2, CODE_GOAL); add_obj(G, T_GOAL, 15, S - 2, S - 2); return; }
    for (int i = 1; i < S - 1; i++) put(G, mid, i, CODE_WALL);
    if (nr == 3) for (int i = 1; i < mid; i++) put(G, i, mid, CODE_WALL);
    if (nr == 4) for (int i = 1; i < S - 1; i++) put(G, i, mid, CODE_WALL);
    const int ndoors = nr == 2 ? 1 : nr;
    const bool ado = G.all_doors_open;
    const uint32_t dinfo = P.dinfo;
    uint32_t oc = 0x3FFFFu;    // obj_choice: bit = type_slot*6 + colour-name (key, ball, box)
#pragma unroll 1
    for (int d = 0; d < ndoors; d++) {                           // a locked door's key (or key box) leaves the list
        const uint32_t di = dinfo >> (8 * d);
        const int col = di & 7;
        if ((di >> 3) & 1) { oc &= ~(1u << col); if ((di >> 4) & 1) oc &= ~(1u << (12 + col)); }
    }
    GSTAMP(G, 11);                                               // walls + door colour/lock draws
#pragma unroll 1
    for (int d = 0; d < ((MGX_GEN_SKIP & 2) ? 0 : ndoors); d++) {
        bool horiz; int lo, hi;
        door_geom(nr, d, mid, S, horiz, lo, hi);
        const int v = lo + (int)((P.dpos >> (4 * d)) & 15);
        const int x = horiz ? v : mid, y = horiz ? mid : v;
        const uint32_t di = dinfo >> (8 * d);
        const bool open = ado && ((P.dopen >> d) & 1);
        put_door(G, x, y, (uint8_t)door_code(di & 7, (di >> 3) & 1, open));
        add_obj(G, T_DOOR, di & 7, x, y);
    }
    GSTAMP(G, 12);                                               // door positions
    if (G.abort) return;
    int gx = 1, gy = 1;
    if (MGX_GEN_SKIP & 4) {
        gx = 1; gy = 1; put(G, gx, gy, CODE_GOAL); add_obj(G, T_GOAL, 15, gx, gy); G.ax = S - 2; G.ay = S - 2;
    } else {
        // `while True: goal_pos = place_obj(Goal()); if next2door: grid.set(None); continue` then
        // place_agent() (custom_env.py:653-667, 933-947, 1394-1408) as ONE
        // rejection loop: a lane's draws go to the goal until one is accepted (free, not next to
        // a door), then to the agent (free).  Each lane draws exactly the reference's sequence;
        // the wave no longer waits for its slowest goal before any lane places its agent.
        bool agent = false;
#pragma unroll 1
        for (uint32_t it = 0;; ++it) {
            GCOUNT(G, 22);
            if (it > 2 * PCG_LOOP_LIMIT) { G.err |= 4u; G.ax = 1; G.ay = 1; break; }
            int x, y;
            pcg_cell(G.pcg, S, x, y);
            if (occupied(G, y * S + x)) continue;          // (the agent is not placed yet: G.ax = -1)
            if (agent) { G.ax = x; G.ay = y; break; }
            if (next2door(G, x, y)) continue;              // goal placed then removed: net no-op
            gx = x; gy = y;
            put(G, gx, gy, CODE_GOAL);
            add_obj(G, T_GOAL, 15, gx, gy);
            agent = true;
        }
        G.adir = pcg_integers(G.pcg, 0, 4);
    }
    GSTAMP(G, 13);                                               // goal + agent (PCG64)
    const int gr = room_of(nr, gx, gy, mid), ar = room_of(nr, G.ax, G.ay, mid);
    // object counters: c0 = (left | upper-left), c1 = (right | lower-left, unused by Q1), c2, c3
    const int n_left = G.num_objects / 2, n_right = G.num_objects - n_left;
    int c0, c1, c2, c3;
    if (nr == 2) { c0 = n_left; c1 = n_right; c2 = c3 = 0; }
    else if (nr == 3) { c0 = n_left / 2; c1 = n_left - c0; c2 = n_right; c3 = 0; }
    else { c0 = n_left / 2; c1 = n_left - c0; c2 = n_right / 2; c3 = n_right - c2; }
    // Per room: which keys it gets (locked doors only) and how many objects (custom_env's
    // decrement of the room counter by its keys and the goal; Q1: the lower-left room
    // of the 3/4-room layouts loops over the upper-left counter).  No RNG involved.
    uint32_t keymask = 0;   // room r: bit 2r = key A placed, bit 2r+1 = key B placed
    uint32_t npack = 0;     // room r: byte r = objects to place (clamped at 0)
    uint32_t kspec = 0;     // room r: bits 4r..4r+3 = door of key A, key B (2 bits each); bit 16+r = chk
#pragma unroll
    for (int r = 0; r < 4; r++) {
        int kA, kB;
        bool chk;
        key_spec(nr, r, ar, kA, kB, chk);
        kspec |= (uint32_t)(kA & 3) << (4 * r) | (uint32_t)(kB & 3) << (4 * r + 2) | (uint32_t)chk << (16 + r);
        const bool a = r < nr && kA >= 0 && ((dinfo >> (8 * kA + 3)) & 1);
        const bool b = r < nr && kB >= 0 && ((dinfo >> (8 * kB + 3)) & 1);
        keymask |= (uint32_t)a << (2 * r) | (uint32_t)b << (2 * r + 1);
        const int ndec = (int)a + (int)b + (int)(gr == r);
        int n;
        if (r == 0) { c0 -= ndec; n = c0; }
        else if (r == 1) { c1 -= ndec; n = (nr == 2) ? c1 : c0; }
        else if (r == 2) { c2 -= ndec; n = c2; }
        else { c3 -= ndec; n = c3; }
        npack |= (uint32_t)(n > 0 ? n : 0) << (8 * r);
    }
    // The keys and objects of all rooms as ONE task sequence: every outer iteration places
    // one key or object for every lane, whatever room/task the lane is at (lanes do not wait
    // for each other at room boundaries).  Each lane still draws exactly the reference's
    // sequence:  for room r: [key A] [key B] then n_r x { choice(obj_choice); position loop }.
    // The rejection loop `while True: p = (randint(x0,x1), randint(y0,y1)); if ok(p): break`
    // is the tight inner loop: the cells a placement must avoid are one precomputed bit set,
    // so a rejected draw costs two SWAR randbelow and one bit test -- the lanes that need many
    // draws (the wave waits for them) no longer re-run the task set-up per draw.
    uint64_t reps = 0;                       // bit y*S of every row y (S <= 8): room masks by multiply
    if (NW == 1)
        for (int i = 0; i < S; i++) reps |= 1ull << (i * S);
    // The task sequence as one 64-bit set, consumed lowest bit first: room r owns bits 16r..16r+15,
    // bit 0 of a room = key A, bit 1 = key B, bits 2.. = its objects (<= 9, num_objects <= 18).
    // Advancing is `todo &= todo - 1` (a per-lane walk over rooms / phases was a divergent loop).
    uint64_t todo = 0;
#pragma unroll
    for (int rr = 0; rr < 4; rr++)
        todo |= (uint64_t)(((keymask >> (2 * rr)) & 3u) | ((((1u << ((npack >> (8 * rr)) & 0xFF)) - 1u) & 0x3FFFu) << 2))
                << (16 * rr);
    if (MGX_GEN_SKIP & 1) return;
    int kx = -1, ky = -1;                    // this room's key A (key B avoids it)
#pragma unroll 1
    while (todo) {
        GCOUNT(G, 20);
        GSTAMP(G, 19);                                           // (commit + task advance of the previous)
        GSTAMP(G, 16);                                           // MT window top-up
        const int slot = (int)__builtin_ctzll(todo);
        const int r = slot >> 4, phase = min(slot & 15, 2);     // 0 key A, 1 key B, 2 object
        int x0, x1, y0, y1;
        room_rect(nr, r, mid, S, x0, x1, y0, y1);
        const bool is_key = phase < 2;
        int cname, ot = T_KEY, ox = -1, oy = -1;
        bool chk = false, kib = false;
        if (is_key) {
            chk = (kspec >> (16 + r)) & 1;
            const uint32_t di = dinfo >> (8 * ((kspec >> (4 * r + 2 * phase)) & 3));
            cname = di & 7;
            kib = (di >> 4) & 1;
            if (phase == 1 && ((keymask >> (2 * r)) & 1)) { ox = kx; oy = ky; }   // key A came just before
        } else {
            if (oc == 0) { G.err |= 8u; break; }
            // the object's random.choice(obj_choice) is the first draw of its placement's rejection loop's
            // first pass (draw_cell has_c); the type and colour are taken once the cell is drawn
        }
        const bool has_c = !is_key && !(MGX_GEN_SKIP & 32);
        const RbConst kc_ = rb_const(is_key ? 1u : (uint32_t)__popc(oc));
        int choice = 0;
        // cells this placement rejects: key -> goal, [agent], [the other key], next to a door;
        // object -> occupied, agent, next to a door
        const int ex0 = is_key ? gx : G.ax, ey0 = is_key ? gy : G.ay;
        const int ex1 = (is_key && !chk) ? -1 : G.ax, ey1 = (is_key && !chk) ? -1 : G.ay;
        const RbConst kx_ = rb_const((uint32_t)(x1 - x0 + 1)), ky_ = rb_const((uint32_t)(y1 - y0 + 1));
        int x, y;
        GSTAMP(G, 17);                                           // task set-up, choice, satisfiability
        if constexpr (NW <= 2) {
            Bits<NW> bad = G.dn;
            if (!is_key) { bad.w0 |= G.occ.w0; if (NW > 1) bad.w1 |= G.occ.w1; }
            bad.set(ey0 * S + ex0);
            if (ex1 >= 0) bad.set(ey1 * S + ex1);
            if (ox >= 0) bad.set(oy * S + ox);
            // no acceptable cell in the room: the reference's loop never ends -> live-lock policy
            // at once (same end state as after the word cap)
            bool sat;
            if constexpr (NW == 1) {
                const uint64_t rows = reps & (((1ull << ((y1 + 1) * S)) - 1ull) & ~((1ull << (y0 * S)) - 1ull));
                sat = ((rows * (uint64_t)(((1u << (x1 - x0 + 1)) - 1u) << x0)) & ~bad.w0) != 0;
            } else {
                sat = rect_has_free(G, x0, x1, y0, y1, !is_key, ex0, ey0, ex1, ey1, ox, oy);
            }
            if (!sat) {
                // no acceptable cell: the reference's loop never ends -> live-lock policy at once (the choice
                // draw before it changes nothing: the attempt's cursor jumps to its cap either way)
                live_lock(G);
                return;
            }
            draw_cell(G, kx_, ky_, x0, y0, x, y, [&](int cx, int cy) { return bad.test(cy * S + cx); },
                      [] { return true; }, has_c, kc_, choice);
            if (G.abort) return;
        } else {
            // S > 11: the cells are tested in the LDS grid; after SAT_PROBE rejections an exhaustive
            // scan of the room decides whether the loop can end (else the live-lock policy)
            const auto bad = [&](int cx, int cy) {
                return (cx == ex0 && cy == ey0) || (cx == ex1 && cy == ey1) || (cx == ox && cy == oy) ||
                       (!is_key && occupied(G, cy * S + cx)) || next2door(G, cx, cy);
            };
            draw_cell(G, kx_, ky_, x0, y0, x, y, bad, [&] {
                for (int xx = x0; xx <= x1; xx++)
                    for (int yy = y0; yy <= y1; yy++)
                        if (!bad(xx, yy)) return true;
                return false;
            }, has_c, kc_, choice);
            if (G.abort) return;
        }
        if (!is_key) {                                           // commit the object's type and colour
            const int b = (MGX_GEN_SKIP & 32) ? __ffs(oc) - 1 : nth_set_bit(oc, choice);
            oc &= ~(1u << b);
            ot = MULTI_TYPES[b / 6];
            cname = b % 6;
        }
        GSTAMP(G, 18);                                           // inner rejection loop
        // commit the placement, then the next task
        const int cidx = cn2idx(cname);
        const int t = is_key ? (kib ? T_BOX : T_KEY) : ot;
        put(G, x, y, mk_code(t, cidx, (is_key && kib) ? 1 : 0));
        add_obj(G, t, cname, x, y, is_key ? OBJ_KEYFLAG : 0u);
        if (phase == 0) { kx = x; ky = y; }
        todo &= todo - 1;
    }
    GSTAMP(G, 14);                                               // keys + objects, room by room
}

template <int NW>
__device__ __forceinline__ int gen_multi(Gen<NW> &G) {             // custom_env.py:595-615
    // [choice([0, 1, 2, 5]) = randbelow(4) when the config names no mission] then randint(2, 4), the doors' draws:
    // the prefix record the refill looked up for this attempt's first word (G.phave: its words already consumed),
    // else drawn here
    const bool draw_cmd = G.cfg_mission < 0;
    Prefix P;
    if (G.phave) {
        pfx_unpack(G.prec, P);
    } else {
#if MGX_GEN_PREFIX2   // diagnostic: the prefix drawn twice (the first discarded): its marginal cost
        { const uint64_t c0_ = G.cur; prefix_draws(G, G.S, draw_cmd, G.all_doors_open != 0, P); G.cur = c0_; G.abort = false; mt_sync(G); }
#endif
        prefix_draws(G, G.S, draw_cmd, G.all_doors_open != 0, P);
        if (G.abort) return 0;
    }
    const int cmd = draw_cmd ? (P.rc == 3 ? 5 : P.rc) : G.cfg_mission;
    GSTAMP(G, 10);                                               // mission + room-count draws
    gen_rooms(G, P);
    return cmd;
}

__device__ const int GTO_T[4] = {T_KEY, T_BALL, T_BOX, T_DOOR};   // self.obj_types
__device__ const int GTG_T[4] = {T_BOX, T_DOOR, T_KEY, T_BALL};
__device__ const int OPN_T[2] = {T_BOX, T_DOOR};
__device__ const int PKP_T[3] = {T_KEY, T_BOX, T_BALL};

// EXT = the generator variant with the problems / features no shipped config uses (full, drp,
// mov, obstacles): compiled out of the default variant so its register budget is unchanged.
template <int NW, bool EXT>
__device__ __forceinline__ int gen_single(Gen<NW> &G) {           // custom_env.py:332-593
    const int *types;
    int ntypes, cmd;
    bool goal = false;
    const bool full = EXT && G.problem == 1;
    if constexpr (EXT) {
        switch (G.problem) {
            case 1: types = GTO_T; ntypes = 4; cmd = -1; goal = true; break;  // full: every (type, colour)
            case 2: types = GTO_T; ntypes = 4; cmd = 0; break;              // gto -> 'go to'
            case 3: types = GTG_T; ntypes = 4; cmd = 5; goal = true; break;  // gtg -> 'go to goal'
            case 4: types = OPN_T; ntypes = 2; cmd = 1; break;              // opn -> 'toggle'
            case 6: types = GTO_T; ntypes = 4; cmd = 3; goal = true; break;  // drp -> 'drop'
            case 7: types = GTO_T; ntypes = 4; cmd = 4; break;              // mov -> 'move <dir>'
            default: types = PKP_T; ntypes = 3; cmd = 2; break;             // pkp -> 'pick up'
        }
    } else {
        switch (G.problem) {
            case 2: types = GTO_T; ntypes = 4; cmd = 0; break;
            case 3: types = GTG_T; ntypes = 4; cmd = 5; goal = true; break;
            case 4: types = OPN_T; ntypes = 2; cmd = 1; break;
            default: types = PKP_T; ntypes = 3; cmd = 2; break;
        }
    }
    uint32_t oc = (1u << (ntypes * 6)) - 1u;
    const int nplace = full ? 24 : G.num_objects;
    for (int k = 0; k < nplace; k++) {
        if (oc == 0) { G.err |= 8u; break; }
        // full: `for objType in obj_types: for objColor in COLOR_NAMES` (no MT draw);
        // else `choice(obj_choice); obj_choice.remove(...)`
        const int b = full ? k : mask_choice(G, oc);
        if (G.abort) return 0;
        oc &= ~(1u << b);
        const int t = types[b / 6], cname = b % 6;
        int x, y;
        draw_free_cell(G, x, y);
        put(G, x, y, mk_code(t, cn2idx(cname), 0));
        add_obj(G, t, cname, x, y);
    }
    if (goal) {
        int x, y;
        draw_free_cell(G, x, y);
        put(G, x, y, CODE_GOAL);
        add_obj(G, T_GOAL, 15, x, y);
    }
    place_agent(G);
    if (full) cmd = pcg_integers(G.pcg, 0, 6);                     // np_random.choice(self.msn_commands)
    return cmd;
}

struct ResetOut {
    uint8_t tx, ty, ta, mission_id;
    int livelocks;
    uint64_t range;        // 'move' target_range (move_range), 0 otherwise
};

// `obj_pos in [o[2] for o in objs]` (the objs list lives in LDS)
template <int NW>
__device__ __forceinline__ bool in_objs(const Gen<NW> &G, int x, int y) {
    const uint32_t key = (uint32_t)x << 8 | (uint32_t)y << 16;
    bool hit = false;
    for (int k = 0; k < G.nobjs; k++) hit |= (G.objs[k] & 0xFFFF00u) == key;
    return hit;
}

// Obstacles (custom_env.py:154-172), after the generator, before the mission target.
//   multi:  while True: p=(randint(1,S-2), randint(1,S-2)); skip the middle row/column;
//           skip p in objs; break if p != agent and not next2door(p)  -> put_obj(Lava())
//   single: place_obj(choice([Lava(), Wall()]))
template <int NW>
__device__ __forceinline__ void place_obstacles(Gen<NW> &G) {
    const int S = G.S, mid = S / 2;
#pragma unroll 1
    for (int k = 0; k < G.n_obstacles; k++) {
        if (G.problem == 0) {
            int x, y, rej = 0;
            for (;;) {
                x = randint(G, 1, S - 2);
                y = randint(G, 1, S - 2);
                if (G.abort) return;
                const bool bad = x == mid || y == mid || in_objs(G, x, y) || (x == G.ax && y == G.ay) ||
                                 next2door(G, x, y);
                if (!bad) break;
                if (++rej == SAT_PROBE) {            // provably unsatisfiable loop -> live-lock policy
                    bool sat = false;
                    for (int xx = 1; xx <= S - 2 && !sat; xx++)
                        for (int yy = 1; yy <= S - 2 && !sat; yy++)
                            sat = !(xx == mid || yy == mid || in_objs(G, xx, yy) || (xx == G.ax && yy == G.ay) ||
                                    next2door(G, xx, yy));
                    if (!sat) { live_lock(G); return; }
                }
            }
            put(G, x, y, CODE_LAVA);
        } else {
            const bool lava = randbelow(G, 2) == 0;
            if (G.abort) return;
            int x, y;
            draw_free_cell(G, x, y);
            put(G, x, y, lava ? CODE_LAVA : CODE_WALL);
        }
    }
}

// 'move' target_range (custom_env.py:219-256): per row (left/right) or column (up/down)
// k = 1..S-2, the first None cell scanning inward from that edge, if any.  Packed as
// bits 0-1 = direction, bits 4k..4k+3 = that cell's x (rows) or y (columns), 0 = none.
template <int NW>
__device__ __forceinline__ uint64_t move_range(const Gen<NW> &G, int d) {
    const int S = G.S;
    uint64_t rg = (uint64_t)d;
    for (int k = 1; k < S - 1; k++) {
        int v;
        bool ok;
        if (d == 0) { v = 1; while (v < S - 1 && G.g[k * S + v] != CODE_EMPTY) v++; ok = v < S - 1; }
        else if (d == 1) { v = S - 2; while (v > 0 && G.g[k * S + v] != CODE_EMPTY) v--; ok = v > 0; }
        else if (d == 2) { v = 1; while (v < S - 1 && G.g[v * S + k] != CODE_EMPTY) v++; ok = v < S - 1; }
        else { v = S - 2; while (v > 0 && G.g[v * S + k] != CODE_EMPTY) v--; ok = v > 0; }
        if (ok) rg |= (uint64_t)v << (4 * k);
    }
    return rg;
}
// agent_pos in target_range
__device__ __forceinline__ bool in_move_range(uint64_t rg, int ax, int ay) {
    const bool rows = (rg & 3) < 2;
    const int idx = rows ? ay : ax, coord = rows ? ax : ay;
    const int ent = (int)((rg >> (4 * idx)) & 15);
    return ent != 0 && ent == coord;
}

// Grid.process_vis(agent_pos=(3, 6)) + Grid.encode(vis_mask) (see_through_walls=False) on a
// rendered frame (fr[c] type, fr[49+c] colour, fr[98+c] state, c = vx*7 + vy): cells the
// agent cannot see become (0, 0, 0).  Bit-parallel over a view row (bit = vx): the
// reference's left-to-right pass sets cell i+1 from a visible see-through cell i, i.e. the
// closure of x |= (x & T) << 1; both passes also light cells i, i+1 (i-1, i) of the row
// above.  The agent cell holds the carried object here, but the world cell under the
// agent is always see-through (it can overlap it), as is any carried object.
__device__ __forceinline__ void apply_vis(uint8_t *fr) {
    uint32_t T[7];
#pragma unroll
    for (int vy = 0; vy < 7; vy++) {
        uint32_t t = 0;
#pragma unroll
        for (int vx = 0; vx < 7; vx++) {
            const int c = vx * 7 + vy;
            const int ty = fr[c], st = fr[98 + c];
            const bool opaque = ty == T_WALL || (ty == T_DOOR && st != 0);   // see_behind() false
            t |= (uint32_t)!opaque << vx;
        }
        T[vy] = t;
    }
    uint64_t vis = 0;
    uint32_t m = 1u << 3;                    // mask[3][6] = True
#pragma unroll
    for (int j = 6; j >= 0; j--) {
        const uint32_t t = T[j];
        uint32_t x = m;
#pragma unroll
        for (int k = 0; k < 6; k++) x |= (x & t & 0x3Fu) << 1;     // for i in range(0, 6)
        const uint32_t s1 = x & t & 0x3Fu;
        uint32_t up = (s1 << 1) | s1;
#pragma unroll
        for (int k = 0; k < 6; k++) x |= (x & t & 0x7Eu) >> 1;     // for i in reversed(range(1, 7))
        const uint32_t s2 = x & t & 0x7Eu;
        up |= (s2 >> 1) | s2;
#pragma unroll
        for (int vx = 0; vx < 7; vx++) vis |= (uint64_t)((x >> vx) & 1u) << (vx * 7 + j);
        m = up;
    }
#pragma unroll
    for (int c = 0; c < 49; c++)
        if (!((vis >> c) & 1ull)) { fr[c] = 0; fr[49 + c] = 0; fr[98 + c] = 0; }
}

template <int NW>
__device__ __forceinline__ void gen_init(Gen<NW> &G) {}

// One attempt of MiniGridEnv.reset -> PlaygroundEnv._gen_grid (custom_env.py:122-267).
// MULTI: the problem is known to be 'multi' (every BASELINE config): the single-room generators
// are not compiled in, which keeps the kernel's code and register allocation to the multi path.
template <int NW, bool EXT, bool MULTI = false>
__device__ __forceinline__ void gen_attempt(Gen<NW> &G, ResetOut &R) {
    const int S = G.S;
    {   // Grid(W, H) of None + wall_rect(0, 0, W, H); the row is 4-B aligned in LDS
        uint32_t *g32 = reinterpret_cast<uint32_t *>(G.g);
        if (NW == 1 && S == 8) {                                  // two dwords per row: 16 constant stores
            constexpr uint32_t W4 = 0x01010101u * CODE_WALL;
            constexpr uint32_t L4 = 0x01010100u * CODE_EMPTY | CODE_WALL, R4 = 0x00010101u * CODE_EMPTY | (uint32_t)CODE_WALL << 24;
            g32[0] = W4; g32[1] = W4; g32[14] = W4; g32[15] = W4;
#pragma unroll
            for (int r = 1; r < 7; r++) { g32[2 * r] = L4; g32[2 * r + 1] = R4; }
        } else {
            const int nw = (S * S + 3) >> 2;
            for (int i = 0; i < nw; i++) g32[i] = 0x01010101u * CODE_EMPTY;
            for (int i = 0; i < S; i++) {
                G.g[i] = CODE_WALL; G.g[(S - 1) * S + i] = CODE_WALL;
                G.g[i * S] = CODE_WALL; G.g[i * S + S - 1] = CODE_WALL;
            }
        }
    }
    G.occ.clear();                                                // wall_rect(0, 0, W, H)
    if constexpr (NW == 1) {                                      // the border as one mask
        const uint64_t row = (1ull << S) - 1ull;
        uint64_t col = 0;
        for (int i = 0; i < S; i++) col |= 1ull << (i * S);
        G.occ.w0 = row | (row << ((S - 1) * S)) | col | (col << (S - 1));
    } else {
        for (int i = 0; i < S; i++) {
            G.occ.set(i); G.occ.set((S - 1) * S + i);
            G.occ.set(i * S); G.occ.set(i * S + S - 1);
        }
    }
    G.dn.clear();
    G.ax = -1; G.ay = -1; G.adir = 0; G.nobjs = 0; G.tmask = 0;
    G.goalx = -1; G.goaly = -1;
    GSTAMP(G, 9);                                                 // attempt setup (mt_sync, grid clear)
    int cmd;
    if constexpr (MULTI) cmd = gen_multi(G);
    else cmd = G.problem == 0 ? gen_multi(G) : gen_single<NW, EXT>(G);
    if (G.abort) return;
    if (EXT && G.n_obstacles) {
        place_obstacles(G);
        if (G.abort) return;
    }
    // the mission's target as locals, R written once (per-branch stores to R's fields were merged
    // through pointer selects, which put R on the stack)
    uint32_t tx = NONE8, ty = NONE8, ta = NONE8, mid = CMD_GOTOGOAL;
    uint64_t range = 0;
    if (EXT && cmd == 3) {                                        // 'drop'
        ta = A_DROP; mid = MID_DROP;
    } else if (EXT && cmd == 4) {                                 // 'move <dir>'
        const int d = pcg_integers(G.pcg, 0, 4);                  // np_random.choice(self.msn_directions)
        range = move_range(G, d);
        mid = MID_MOVE + d;
    } else if (cmd == 0) {                                               // 'go to' (np_random.integers)
        int i = 0;
        uint32_t bad = 0;
        for (uint32_t it = 0;; ++it) {
            if (it > PCG_LOOP_LIMIT) { bad = 4u; break; }
            i = pcg_integers(G.pcg, 0, G.nobjs);
            if ((G.objs[i] & 15) != T_GOAL) break;
        }
        G.err |= bad;
        const uint32_t o = G.objs[i];
        tx = (o >> 8) & 0xFF; ty = (o >> 16) & 0xFF; ta = A_DONE;
        mid = CMD_GOTO | (((o >> 4) & 15) << 2) | (type_slot(o & 15) << 5);
    } else if (cmd == 1 || cmd == 2) {                            // 'toggle' / 'pick up' (random.choice)
        const uint32_t want = cmd == 1 ? (1u << T_BOX) | (1u << T_DOOR) : (1u << T_BOX) | (1u << T_KEY) | (1u << T_BALL);
        if (!(G.tmask & want)) { live_lock(G); return; }     // no such object: the reference loops forever
        int i;
        for (;;) {
            i = randbelow(G, (uint32_t)G.nobjs);
            if (G.abort) return;
            if ((want >> (G.objs[i] & 15)) & 1) break;
        }
        const uint32_t o = G.objs[i];
        tx = (o >> 8) & 0xFF; ty = (o >> 16) & 0xFF;
        ta = cmd == 1 ? A_TOGGLE : A_PICKUP;
        mid = (cmd == 1 ? CMD_TOGGLE : CMD_PICKUP) | (((o >> 4) & 15) << 2) | (type_slot(o & 15) << 5);
    } else if (G.goalx >= 0) {                                    // 'go to goal': the first Goal in objs
        tx = (uint32_t)G.goalx;                                   // (recorded by add_obj: no scan of the list)
        ty = (uint32_t)G.goaly;
    }
    R.tx = (uint8_t)tx; R.ty = (uint8_t)ty; R.ta = (uint8_t)ta; R.mission_id = (uint8_t)mid;
    R.range = range;
}

// MiniGridEnv.reset with the engine's live-lock retry policy.
template <int NW, bool EXT>
__device__ __forceinline__ void reset_env(Gen<NW> &G, ResetOut &R) {
    R.livelocks = 0;
    for (;;) {
        GSTAMP(G, 8);                   // previous episode's copy-out + loop
        G.astart = G.cur;
        G.abort = false;
        mt_sync(G);                     // register queue at the attempt's first word
        gen_attempt<NW, EXT>(G, R);
        GSTAMP(G, 15);                  // mission target selection
        if (!G.abort) break;
        R.livelocks++;
        if (R.livelocks > 100000) { G.err |= 4u; break; }
    }
}

}  // namespace mgx
