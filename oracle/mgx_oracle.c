/*
 * mgx_oracle.c -- CPU restatement of the reference's MiniGrid hot path.
 *
 * TEST INFRASTRUCTURE / CHECKER ONLY.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg load this (via oracle/oracle.py).  The
 * product path (minigrid-rl_amd/) never links or calls it.
 *
 * What it restates, function by function (file:line into /root/reference):
 *   PlaygroundEnv._gen_grid            src/custom_env.py:122-267
 *   PlaygroundEnv.step                 src/custom_env.py:269-330
 *   obstacles (cfg.obstacles)          src/custom_env.py:154-172
 *   'move' target_range                src/custom_env.py:219-256
 *   _generate_full_map                 src/custom_env.py:332-369
 *   _generate_{gto,gtg,open,pkp}_map   src/custom_env.py:371-513
 *   _generate_{drop,move}_map          src/custom_env.py:515-593
 *   _generate_multi_map                src/custom_env.py:595-615
 *   _generate_2_rooms                  src/custom_env.py:617-855
 *   _generate_3_rooms                  src/custom_env.py:857-1297
 *   _generate_4_rooms                  src/custom_env.py:1299-2034
 *   next2door                          src/custom_env.py:2036-2046
 *   TokenizeVocabWrapper               src/environment.py:69-112
 *   Discrete2BoxWrapper                src/environment.py:138-149
 * and the third-party semantics they call (not vendored; SURVEY.md App. A,
 * parity unpinned at that boundary): minigrid MiniGridEnv.{reset,step,
 * gen_obs,gen_obs_grid,place_obj,place_agent,put_obj,_reward},
 * Grid.{slice,rotate_left,encode,process_vis}, world objects (see_behind); CPython random (MT19937 init_by_array,
 * getrandbits, _randbelow, choice, randint); numpy SeedSequence + PCG64 +
 * Generator.integers (Lemire32 over the has_uint32-buffered next_uint32);
 * SB3 SubprocVecEnv auto-reset (each env owns an MT19937 seeded cfg.seed).
 *
 * Deliberately structured like the reference (object grid, literal
 * slice + rotate_left observation, per-env MT19937 state) and NOT like the
 * HIP engine (closed-form view, shared MT table + cursor), so that agreement
 * between the two is evidence, not tautology.
 *
 * Live-lock policy (the reference hangs): a reset attempt
 * may consume at most `livelock_words` MT words; the attempt that would draw
 * one more is abandoned and reset re-runs unseeded, streams continuing.
 */
#include <math.h>
#include <setjmp.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;

/* ------------------------------------------------------------------ */
/* CPython random: MT19937 (Modules/_randommodule.c, mt19937ar)         */
/* ------------------------------------------------------------------ */
typedef struct { uint32_t mt[624]; int mti; } mt_t;

static void mt_init_genrand(mt_t *m, uint32_t s) {
    m->mt[0] = s;
    for (int i = 1; i < 624; i++)
        m->mt[i] = 1812433253U * (m->mt[i - 1] ^ (m->mt[i - 1] >> 30)) + (uint32_t)i;
    m->mti = 624;
}

static void mt_init_by_array(mt_t *m, const uint32_t *key, int klen) {
    mt_init_genrand(m, 19650218U);
    int i = 1, j = 0;
    int k = 624 > klen ? 624 : klen;
    for (; k; k--) {
        m->mt[i] = (m->mt[i] ^ ((m->mt[i - 1] ^ (m->mt[i - 1] >> 30)) * 1664525U)) + key[j] + (uint32_t)j;
        i++; j++;
        if (i >= 624) { m->mt[0] = m->mt[623]; i = 1; }
        if (j >= klen) j = 0;
    }
    for (k = 623; k; k--) {
        m->mt[i] = (m->mt[i] ^ ((m->mt[i - 1] ^ (m->mt[i - 1] >> 30)) * 1566083941U)) - (uint32_t)i;
        i++;
        if (i >= 624) { m->mt[0] = m->mt[623]; i = 1; }
    }
    m->mt[0] = 0x80000000U;
}

static uint32_t mt_next(mt_t *m) {
    static const uint32_t mag01[2] = {0U, 0x9908b0dfU};
    uint32_t y;
    if (m->mti >= 624) {
        int kk;
        for (kk = 0; kk < 624 - 397; kk++) {
            y = (m->mt[kk] & 0x80000000U) | (m->mt[kk + 1] & 0x7fffffffU);
            m->mt[kk] = m->mt[kk + 397] ^ (y >> 1) ^ mag01[y & 1U];
        }
        for (; kk < 623; kk++) {
            y = (m->mt[kk] & 0x80000000U) | (m->mt[kk + 1] & 0x7fffffffU);
            m->mt[kk] = m->mt[kk + (397 - 624)] ^ (y >> 1) ^ mag01[y & 1U];
        }
        y = (m->mt[623] & 0x80000000U) | (m->mt[0] & 0x7fffffffU);
        m->mt[623] = m->mt[396] ^ (y >> 1) ^ mag01[y & 1U];
        m->mti = 0;
    }
    y = m->mt[m->mti++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680U;
    y ^= (y << 15) & 0xefc60000U;
    y ^= (y >> 18);
    return y;
}

/* random.seed(n) for a non-negative int n: init_by_array(32-bit chunks). */
static void mt_seed_int(mt_t *m, uint64_t n) {
    uint32_t key[2];
    int klen = 0;
    if (n == 0) key[klen++] = 0;
    while (n) { key[klen++] = (uint32_t)(n & 0xffffffffU); n >>= 32; }
    mt_init_by_array(m, key, klen);
}

/* ------------------------------------------------------------------ */
/* numpy SeedSequence (bit_generator.pyx) + PCG64 (pcg64.h/.c)          */
/* ------------------------------------------------------------------ */
#define SS_INIT_A 0x43b0d7e5U
#define SS_MULT_A 0x931e8875U
#define SS_INIT_B 0x8b51f9ddU
#define SS_MULT_B 0x58f38dedU
#define SS_MIX_L 0xca01f9ddU
#define SS_MIX_R 0x4973f715U

static uint32_t ss_hashmix(uint32_t v, uint32_t *hc) {
    v ^= *hc;
    *hc *= SS_MULT_A;
    v *= *hc;
    v ^= v >> 16;
    return v;
}
static uint32_t ss_mix(uint32_t x, uint32_t y) {
    uint32_t r = SS_MIX_L * x - SS_MIX_R * y;
    r ^= r >> 16;
    return r;
}

/* SeedSequence(seed).generate_state(4, uint64) for 0 <= seed < 2^64. */
static void seedseq_u64x4(uint64_t seed, uint64_t out[4]) {
    uint32_t ent[2];
    int nent = 0;
    if (seed == 0) ent[nent++] = 0;
    while (seed) { ent[nent++] = (uint32_t)(seed & 0xffffffffU); seed >>= 32; }
    uint32_t pool[4];
    uint32_t hc = SS_INIT_A;
    for (int i = 0; i < 4; i++) pool[i] = ss_hashmix(i < nent ? ent[i] : 0U, &hc);
    for (int s = 0; s < 4; s++)
        for (int d = 0; d < 4; d++)
            if (s != d) pool[d] = ss_mix(pool[d], ss_hashmix(pool[s], &hc));
    /* (entropy longer than the pool: not reachable for < 2^128 seeds) */
    uint32_t w[8];
    uint32_t hb = SS_INIT_B;
    for (int i = 0; i < 8; i++) {
        uint32_t v = pool[i & 3];
        v ^= hb;
        hb *= SS_MULT_B;
        v *= hb;
        v ^= v >> 16;
        w[i] = v;
    }
    for (int i = 0; i < 4; i++) out[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
}

typedef struct {
    u128 state, inc;
    int has_uint32;
    uint32_t uinteger;
} pcg_t;

static const u128 PCG_MULT = (((u128)2549297995355413924ULL) << 64) | (u128)4865540595714422341ULL;

static void pcg_step(pcg_t *p) { p->state = p->state * PCG_MULT + p->inc; }

static void pcg_seed(pcg_t *p, uint64_t seed) {
    uint64_t v[4];
    seedseq_u64x4(seed, v);
    u128 initstate = ((u128)v[0] << 64) | v[1];
    u128 initseq = ((u128)v[2] << 64) | v[3];
    p->state = 0;
    p->inc = (initseq << 1) | 1;
    pcg_step(p);
    p->state += initstate;
    pcg_step(p);
    p->has_uint32 = 0;
    p->uinteger = 0;
}

static uint64_t pcg_next64(pcg_t *p) {
    pcg_step(p);
    uint64_t hi = (uint64_t)(p->state >> 64), lo = (uint64_t)p->state;
    unsigned rot = (unsigned)(p->state >> 122);
    uint64_t x = hi ^ lo;
    return (x >> rot) | (x << ((64 - rot) & 63));
}

static uint32_t pcg_next32(pcg_t *p) {
    if (p->has_uint32) { p->has_uint32 = 0; return p->uinteger; }
    uint64_t n = pcg_next64(p);
    p->has_uint32 = 1;
    p->uinteger = (uint32_t)(n >> 32);
    return (uint32_t)(n & 0xffffffffU);
}

/* Generator.integers(lo, hi) scalar int64 path (random_bounded_uint64 ->
 * buffered_bounded_lemire_uint32 with the bitgen's own 32-bit buffer). */
static int64_t pcg_integers(pcg_t *p, int64_t lo, int64_t hi) {
    uint64_t rng = (uint64_t)(hi - 1 - lo);
    if (rng == 0) return lo;
    if (rng == 0xffffffffULL) return lo + (int64_t)pcg_next32(p);
    uint32_t rng_excl = (uint32_t)rng + 1U;
    uint64_t m = (uint64_t)pcg_next32(p) * rng_excl;
    uint32_t left = (uint32_t)m;
    if (left < rng_excl) {
        uint32_t thr = (uint32_t)(0xffffffffU - (uint32_t)rng) % rng_excl;
        while (left < thr) {
            m = (uint64_t)pcg_next32(p) * rng_excl;
            left = (uint32_t)m;
        }
    }
    return lo + (int64_t)(m >> 32);
}

/* ------------------------------------------------------------------ */
/* minigrid constants / world objects                                  */
/* ------------------------------------------------------------------ */
enum { O_NONE = 0, O_EMPTY = 1, O_WALL = 2, O_DOOR = 4, O_KEY = 5, O_BALL = 6, O_BOX = 7, O_GOAL = 8, O_LAVA = 9 };
enum { A_LEFT = 0, A_RIGHT, A_FORWARD, A_PICKUP, A_DROP, A_TOGGLE, A_DONE };
/* COLOR_NAMES = sorted(COLORS) = blue green grey purple red yellow; index -> COLOR_TO_IDX */
static const int CN2IDX[6] = {2, 1, 5, 3, 0, 4};
static const char *CN_NAME[6] = {"blue", "green", "grey", "purple", "red", "yellow"};
enum { C_RED = 0, C_GREEN = 1, C_GREY = 5 };

typedef struct {
    uint8_t type;   /* O_NONE == Python None */
    uint8_t color;  /* COLOR_TO_IDX */
    uint8_t is_open, is_locked;
    uint8_t contains; /* box: 1 = holds Key(same colour) */
} cell_t;

#define MAXS 32
#define MAXOBJ 64

typedef struct { int type; int cname; int x, y; } objrec_t; /* cname: COLOR_NAMES idx, -1 goal */

enum { P_MULTI = 0, P_FULL, P_GTO, P_GTG, P_OPN, P_PKP, P_DRP, P_MOV };
enum { CMD_GOTO = 0, CMD_TOGGLE = 1, CMD_PICKUP = 2, CMD_DROP = 3, CMD_MOVE = 4, CMD_GOTOGOAL = 5 };
static const char *CMD_NAME[6] = {"go to", "toggle", "pick up", "drop", "move", "go to goal"};

typedef struct {
    int S, max_steps, problem, cfg_mission, num_objects, all_doors_open;
    int see_through_walls, n_obstacles;
    cell_t grid[MAXS * MAXS];
    int ax, ay, adir;
    cell_t carrying; /* type O_NONE == None */
    int step_count;
    int mission_done;
    int has_reward; double reward;
    int has_tpos, tx, ty;
    int target_action; /* -1 == None */
    char mission[64];
    mt_t mt;
    int64_t mt_words, attempt_start, livelock_words;
    pcg_t pcg;
    jmp_buf jb;
    objrec_t objs[MAXOBJ]; int nobjs;
    int range_x[MAXS * 2], range_y[MAXS * 2], nrange;   /* self.target_range */
    int manual;     /* PlaygroundEnv(manual=True) (custom_env.py:325): 'done' ends only a completed mission */
} env_t;

typedef struct {
    int n;
    env_t *e;
} orc_vec;

/* ---------------- RNG front-ends used by the reference --------------- */
static uint32_t mt_word(env_t *e) {
    if (e->mt_words - e->attempt_start >= e->livelock_words) longjmp(e->jb, 1);
    e->mt_words++;
    return mt_next(&e->mt);
}
static int bitlen(uint32_t n) { int k = 0; while (n) { k++; n >>= 1; } return k; }
static int randbelow(env_t *e, int n) {           /* Random._randbelow_with_getrandbits */
    int k = bitlen((uint32_t)n);
    uint32_t r = mt_word(e) >> (32 - k);
    while (r >= (uint32_t)n) r = mt_word(e) >> (32 - k);
    return (int)r;
}
static int randint(env_t *e, int a, int b) { return a + randbelow(e, b - a + 1); }
static int rint_np(env_t *e, int lo, int hi) { return (int)pcg_integers(&e->pcg, lo, hi); }

/* ---------------- grid ------------------------------------------------ */
static cell_t *G(env_t *e, int x, int y) { return &e->grid[y * e->S + x]; }
static void gset(env_t *e, int x, int y, cell_t c) { *G(e, x, y) = c; }
static cell_t mk(int type, int color) { cell_t c = {(uint8_t)type, (uint8_t)color, 0, 0, 0}; return c; }
static cell_t mk_none(void) { return mk(O_NONE, 0); }
static cell_t mk_wall(void) { return mk(O_WALL, C_GREY); }
static cell_t mk_goal(void) { return mk(O_GOAL, C_GREEN); }
static cell_t mk_lava(void) { return mk(O_LAVA, C_RED); }
static cell_t mk_door(int cname, int locked, int open) {
    cell_t c = mk(O_DOOR, CN2IDX[cname]); c.is_locked = (uint8_t)locked; c.is_open = (uint8_t)open; return c;
}
static cell_t mk_box_key(int cname) { cell_t c = mk(O_BOX, CN2IDX[cname]); c.contains = 1; return c; }

static void encode_cell(const cell_t *c, uint8_t out[3]) {
    if (c->type == O_NONE) { out[0] = O_EMPTY; out[1] = 0; out[2] = 0; return; }
    out[0] = c->type; out[1] = c->color; out[2] = 0;
    if (c->type == O_DOOR) out[2] = c->is_open ? 0 : (c->is_locked ? 2 : 1);
}

static int can_overlap(const cell_t *c) {
    return c->type == O_GOAL || c->type == O_LAVA || (c->type == O_DOOR && c->is_open);
}
static int see_behind(const cell_t *c) { return c->type == O_WALL ? 0 : (c->type == O_DOOR ? c->is_open : 1); }
static int can_pickup(const cell_t *c) { return c->type == O_KEY || c->type == O_BALL || c->type == O_BOX; }

static int next2door(env_t *e, int x, int y) {
    return G(e, x - 1, y)->type == O_DOOR || G(e, x + 1, y)->type == O_DOOR ||
           G(e, x, y - 1)->type == O_DOOR || G(e, x, y + 1)->type == O_DOOR;
}

/* MiniGridEnv.place_obj(obj) over the whole grid; returns pos. */
static void place_obj(env_t *e, cell_t obj, int *px, int *py) {
    for (;;) {
        int x = rint_np(e, 0, e->S);
        int y = rint_np(e, 0, e->S);
        if (G(e, x, y)->type != O_NONE) continue;
        if (x == e->ax && y == e->ay) continue;
        gset(e, x, y, obj);
        *px = x; *py = y;
        return;
    }
}
static void place_agent(env_t *e) {
    e->ax = -1; e->ay = -1;
    int x, y;
    place_obj(e, mk_none(), &x, &y);
    e->ax = x; e->ay = y;
    e->adir = rint_np(e, 0, 4);
}

static void add_obj(env_t *e, int type, int cname, int x, int y) {
    objrec_t *o = &e->objs[e->nobjs++];
    o->type = type; o->cname = cname; o->x = x; o->y = y;
}
static int in_objs(env_t *e, int x, int y) {
    for (int i = 0; i < e->nobjs; i++) if (e->objs[i].x == x && e->objs[i].y == y) return 1;
    return 0;
}

/* ------------------- ordered "list" of (type, cname) ----------------- */
typedef struct { int type[32], cname[32]; int n; } olist_t;
static void ol_init(olist_t *l, const int *types, int ntypes) {
    l->n = 0;
    for (int t = 0; t < ntypes; t++)
        for (int c = 0; c < 6; c++) { l->type[l->n] = types[t]; l->cname[l->n] = c; l->n++; }
}
static void ol_remove(olist_t *l, int type, int cname) {  /* list.remove: first match, ValueError if absent */
    for (int i = 0; i < l->n; i++)
        if (l->type[i] == type && l->cname[i] == cname) {
            for (int j = i; j + 1 < l->n; j++) { l->type[j] = l->type[j + 1]; l->cname[j] = l->cname[j + 1]; }
            l->n--;
            return;
        }
    fprintf(stderr, "oracle: list.remove(x): x not in list\n");
    abort();
}
static void ol_choice(env_t *e, olist_t *l, int *type, int *cname) {
    int i = randbelow(e, l->n);
    *type = l->type[i]; *cname = l->cname[i];
}

typedef struct { int c[6]; int n; } clist_t;
static void cl_init(clist_t *l) { for (int i = 0; i < 6; i++) l->c[i] = i; l->n = 6; }
static int cl_choice_remove(env_t *e, clist_t *l) {
    int i = randbelow(e, l->n);
    int v = l->c[i];
    for (int j = i; j + 1 < l->n; j++) l->c[j] = l->c[j + 1];
    l->n--;
    return v;
}

static int choice_bool(env_t *e) { return randbelow(e, 2) == 0; } /* choice([True, False]) */

/* --------------------------- room generators -------------------------- */
/* Shared blocks, each a literal restatement of a repeated reference block. */

/* `while True: p=(randint(x0,x1), randint(y0,y1)); if p!=goal and [p!=agent]
 *  and [p!=other] and not next2door(p): break` then grid.set Box/Key, objs.append */
static void place_key(env_t *e, int x0, int x1, int y0, int y1, int gx, int gy,
                      int check_agent, int ox, int oy, int cname, int key_in_box,
                      int *kx, int *ky) {
    int x, y;
    for (;;) {
        x = randint(e, x0, x1);
        y = randint(e, y0, y1);
        if (x == gx && y == gy) continue;
        if (check_agent && x == e->ax && y == e->ay) continue;
        if (ox >= 0 && x == ox && y == oy) continue;
        if (next2door(e, x, y)) continue;
        break;
    }
    if (key_in_box) { gset(e, x, y, mk_box_key(cname)); add_obj(e, O_BOX, cname, x, y); }
    else { gset(e, x, y, mk(O_KEY, CN2IDX[cname])); add_obj(e, O_KEY, cname, x, y); }
    if (kx) { *kx = x; *ky = y; }
}

/* `for _ in range(n): (t,c)=choice(obj_choice); remove; while True: p=...;
 *  for o in objs: if p==o.pos: break / else: if p!=agent and not next2door: break` */
static void place_objects(env_t *e, olist_t *oc, int n, int x0, int x1, int y0, int y1) {
    for (int k = 0; k < n; k++) {
        int t, c;
        ol_choice(e, oc, &t, &c);
        ol_remove(oc, t, c);
        int x, y;
        for (;;) {
            x = randint(e, x0, x1);
            y = randint(e, y0, y1);
            if (in_objs(e, x, y)) continue;
            if (x == e->ax && y == e->ay) continue;
            if (next2door(e, x, y)) continue;
            break;
        }
        gset(e, x, y, mk(t, CN2IDX[c]));
        add_obj(e, t, c, x, y);
    }
}

static void place_goal_multi(env_t *e, int *gx, int *gy) {
    for (;;) {
        place_obj(e, mk_goal(), gx, gy);
        if (next2door(e, *gx, *gy)) { gset(e, *gx, *gy, mk_none()); continue; }
        break;
    }
    add_obj(e, O_GOAL, -1, *gx, *gy);
}

static int door_open_flag(env_t *e) { return e->all_doors_open ? choice_bool(e) : 0; }
static int door_locked_flag(env_t *e) { return e->all_doors_open ? 0 : choice_bool(e); }

static const int MULTI_TYPES[3] = {O_KEY, O_BALL, O_BOX};

static void gen_2_rooms(env_t *e, int mid) {   /* custom_env.py:617-855 */
    int S = e->S;
    int n_left = e->num_objects / 2, n_right = e->num_objects - n_left;
    olist_t oc; ol_init(&oc, MULTI_TYPES, 3);
    for (int i = 1; i < S - 1; i++) gset(e, mid, i, mk_wall());
    clist_t dc; cl_init(&dc);
    int dcol = cl_choice_remove(e, &dc);
    int locked = door_locked_flag(e);
    int kib = choice_bool(e);
    if (locked) { ol_remove(&oc, O_KEY, dcol); if (kib) ol_remove(&oc, O_BOX, dcol); }
    int j = randint(e, 1, S - 2);
    gset(e, mid, j, mk_door(dcol, locked, door_open_flag(e)));
    add_obj(e, O_DOOR, dcol, mid, j);
    int gx, gy; place_goal_multi(e, &gx, &gy);
    int goal_left = gx < mid;
    place_agent(e);
    int agent_left = e->ax < mid;
    if (agent_left && locked) { n_left--; place_key(e, 1, mid - 1, 1, S - 2, gx, gy, 1, -1, -1, dcol, kib, 0, 0); }
    if (goal_left) n_left--;
    place_objects(e, &oc, n_left, 1, mid - 1, 1, S - 2);
    if (!agent_left && locked) { n_right--; place_key(e, mid + 1, S - 2, 1, S - 2, gx, gy, 1, -1, -1, dcol, kib, 0, 0); }
    if (!goal_left) n_right--;
    place_objects(e, &oc, n_right, mid + 1, S - 2, 1, S - 2);
}

static void gen_3_rooms(env_t *e, int mid) {   /* custom_env.py:857-1297 */
    int S = e->S;
    int n_left = e->num_objects / 2;
    int n_lu = n_left / 2, n_ll = n_left - n_lu, n_right = e->num_objects - n_left;
    olist_t oc; ol_init(&oc, MULTI_TYPES, 3);
    for (int i = 1; i < S - 1; i++) gset(e, mid, i, mk_wall());
    for (int i = 1; i < mid; i++) gset(e, i, mid, mk_wall());
    clist_t dc; cl_init(&dc);
    int h_col = cl_choice_remove(e, &dc);
    int h_lk = door_locked_flag(e); int h_kib = choice_bool(e);
    if (h_lk) { ol_remove(&oc, O_KEY, h_col); if (h_kib) ol_remove(&oc, O_BOX, h_col); }
    int vu_col = cl_choice_remove(e, &dc);
    int vu_lk = door_locked_flag(e); int vu_kib = choice_bool(e);
    if (vu_lk) { ol_remove(&oc, O_KEY, vu_col); if (vu_kib) ol_remove(&oc, O_BOX, vu_col); }
    int vl_col = cl_choice_remove(e, &dc);
    int vl_lk = door_locked_flag(e); int vl_kib = choice_bool(e);
    if (vl_lk) { ol_remove(&oc, O_KEY, vl_col); if (vl_kib) ol_remove(&oc, O_BOX, vl_col); }
    int h_i = randint(e, 1, mid - 1);
    gset(e, h_i, mid, mk_door(h_col, h_lk, door_open_flag(e))); add_obj(e, O_DOOR, h_col, h_i, mid);
    int vu_j = randint(e, 1, mid - 1);
    gset(e, mid, vu_j, mk_door(vu_col, vu_lk, door_open_flag(e))); add_obj(e, O_DOOR, vu_col, mid, vu_j);
    int vl_j = randint(e, mid + 1, S - 2);
    gset(e, mid, vl_j, mk_door(vl_col, vl_lk, door_open_flag(e))); add_obj(e, O_DOOR, vl_col, mid, vl_j);
    int gx, gy; place_goal_multi(e, &gx, &gy);
    int goal_left = gx < mid, goal_upper = gy < mid;
    place_agent(e);
    int a_left = e->ax < mid, a_upper = e->ay < mid;
    /* upper left */
    if (a_left && a_upper) {
        int kx = -1, ky = -1;
        if (vu_lk) { n_lu--; place_key(e, 1, mid - 1, 1, mid - 1, gx, gy, 1, -1, -1, vu_col, vu_kib, &kx, &ky); }
        if (h_lk) { n_lu--; place_key(e, 1, mid - 1, 1, mid - 1, gx, gy, 1, kx, ky, h_col, h_kib, 0, 0); }
    }
    if (goal_left && goal_upper) n_lu--;
    place_objects(e, &oc, n_lu, 1, mid - 1, 1, mid - 1);
    /* lower left */
    if (a_left && !a_upper) {
        int kx = -1, ky = -1;
        if (vl_lk) { n_ll--; place_key(e, 1, mid - 1, mid + 1, S - 2, gx, gy, 1, -1, -1, vl_col, vl_kib, &kx, &ky); }
        if (h_lk) { n_ll--; place_key(e, 1, mid - 1, mid + 1, S - 2, gx, gy, 1, kx, ky, h_col, h_kib, 0, 0); }
    }
    if (goal_left && !goal_upper) n_ll--;
    place_objects(e, &oc, n_lu /* Q1: custom_env.py:1119 */, 1, mid - 1, mid + 1, S - 2);
    (void)n_ll;
    /* right */
    if (!a_left) {
        int kx = -1, ky = -1;
        if (vl_lk) { n_right--; place_key(e, mid + 1, S - 2, 1, S - 2, gx, gy, 1, -1, -1, vl_col, vl_kib, &kx, &ky); }
        if (vu_lk) { n_right--; place_key(e, mid + 1, S - 2, 1, S - 2, gx, gy, 1, kx, ky, vu_col, vu_kib, 0, 0); }
    }
    if (!goal_left) n_right--;
    place_objects(e, &oc, n_right, mid + 1, S - 2, 1, S - 2);
}

static void gen_4_rooms(env_t *e, int mid) {   /* custom_env.py:1299-2034 */
    int S = e->S;
    int n_left = e->num_objects / 2;
    int n_lu = n_left / 2, n_ll = n_left - n_lu;
    int n_right = e->num_objects - n_left;
    int n_ru = n_right / 2, n_rl = n_right - n_ru;
    olist_t oc; ol_init(&oc, MULTI_TYPES, 3);
    for (int i = 1; i < S - 1; i++) gset(e, mid, i, mk_wall());
    for (int i = 1; i < S - 1; i++) gset(e, i, mid, mk_wall());
    clist_t dc; cl_init(&dc);
    int hl_col = cl_choice_remove(e, &dc);
    int hl_lk = door_locked_flag(e); int hl_kib = choice_bool(e);
    if (hl_lk) { ol_remove(&oc, O_KEY, hl_col); if (hl_kib) ol_remove(&oc, O_BOX, hl_col); }
    int hr_col = cl_choice_remove(e, &dc);
    int hr_lk = door_locked_flag(e); int hr_kib = choice_bool(e);
    if (hr_lk) { ol_remove(&oc, O_KEY, hr_col); if (hr_kib) ol_remove(&oc, O_BOX, hr_col); }
    int vu_col = cl_choice_remove(e, &dc);
    int vu_lk = door_locked_flag(e); int vu_kib = choice_bool(e);
    if (vu_lk) { ol_remove(&oc, O_KEY, vu_col); if (vu_kib) ol_remove(&oc, O_BOX, vu_col); }
    int vl_col = cl_choice_remove(e, &dc);
    int vl_lk = door_locked_flag(e); int vl_kib = choice_bool(e);
    if (vl_lk) { ol_remove(&oc, O_KEY, vl_col); if (vl_kib) ol_remove(&oc, O_BOX, vl_col); }
    int hl_i = randint(e, 1, mid - 1);
    gset(e, hl_i, mid, mk_door(hl_col, hl_lk, door_open_flag(e))); add_obj(e, O_DOOR, hl_col, hl_i, mid);
    int hr_i = randint(e, mid + 1, S - 2);
    gset(e, hr_i, mid, mk_door(hr_col, hr_lk, door_open_flag(e))); add_obj(e, O_DOOR, hr_col, hr_i, mid);
    int vu_j = randint(e, 1, mid - 1);
    gset(e, mid, vu_j, mk_door(vu_col, vu_lk, door_open_flag(e))); add_obj(e, O_DOOR, vu_col, mid, vu_j);
    int vl_j = randint(e, mid + 1, S - 2);
    gset(e, mid, vl_j, mk_door(vl_col, vl_lk, door_open_flag(e))); add_obj(e, O_DOOR, vl_col, mid, vl_j);
    int gx, gy; place_goal_multi(e, &gx, &gy);
    int goal_left = gx < mid, goal_upper = gy < mid;
    place_agent(e);
    int a_left = e->ax < mid, a_upper = e->ay < mid;
    /* --- upper left room (custom_env.py:1414-1530) --- */
    if (a_left && a_upper) {
        int kx = -1, ky = -1;
        if (vu_lk) { n_lu--; place_key(e, 1, mid - 1, 1, mid - 1, gx, gy, 1, -1, -1, vu_col, vu_kib, &kx, &ky); }
        if (hl_lk) { n_lu--; place_key(e, 1, mid - 1, 1, mid - 1, gx, gy, 1, kx, ky, hl_col, hl_kib, 0, 0); }
    } else if (a_left && !a_upper) {
        if (vu_lk) { n_lu--; place_key(e, 1, mid - 1, 1, mid - 1, gx, gy, 0, -1, -1, vu_col, vu_kib, 0, 0); }
    } else if (!a_left && a_upper) {
        if (hl_lk) { n_lu--; place_key(e, 1, mid - 1, 1, mid - 1, gx, gy, 0, -1, -1, hl_col, hl_kib, 0, 0); }
    }
    if (goal_left && goal_upper) n_lu--;
    place_objects(e, &oc, n_lu, 1, mid - 1, 1, mid - 1);
    /* --- lower left room (custom_env.py:1569-1685) --- */
    if (a_left && !a_upper) {
        int kx = -1, ky = -1;
        if (vl_lk) { n_ll--; place_key(e, 1, mid - 1, mid + 1, S - 2, gx, gy, 1, -1, -1, vl_col, vl_kib, &kx, &ky); }
        if (hl_lk) { n_ll--; place_key(e, 1, mid - 1, mid + 1, S - 2, gx, gy, 1, kx, ky, hl_col, hl_kib, 0, 0); }
    } else if (!a_left && !a_upper) {
        if (hl_lk) { n_ll--; place_key(e, 1, mid - 1, mid + 1, S - 2, gx, gy, 0, -1, -1, hl_col, hl_kib, 0, 0); }
    } else if (a_left && a_upper) {
        if (vl_lk) { n_ll--; place_key(e, 1, mid - 1, mid + 1, S - 2, gx, gy, 0, -1, -1, vl_col, vl_kib, 0, 0); }
    }
    if (goal_left && !goal_upper) n_ll--;
    place_objects(e, &oc, n_lu /* Q1: custom_env.py:1660 */, 1, mid - 1, mid + 1, S - 2);
    (void)n_ll;
    /* --- upper right room (custom_env.py:1724-1841) --- */
    if (!a_left && a_upper) {
        int kx = -1, ky = -1;
        if (vu_lk) { n_ru--; place_key(e, mid + 1, S - 2, 1, mid - 1, gx, gy, 1, -1, -1, vu_col, vu_kib, &kx, &ky); }
        if (hr_lk) { n_ru--; place_key(e, mid + 1, S - 2, 1, mid - 1, gx, gy, 1, kx, ky, hr_col, hr_kib, 0, 0); }
    } else if (!a_left && !a_upper) {
        if (vu_lk) { n_ru--; place_key(e, mid + 1, S - 2, 1, mid - 1, gx, gy, 0, -1, -1, vu_col, vu_kib, 0, 0); }
    } else if (a_left && a_upper) {
        if (hr_lk) { n_ru--; place_key(e, mid + 1, S - 2, 1, mid - 1, gx, gy, 0, -1, -1, hr_col, hr_kib, 0, 0); }
    }
    if (!goal_left && goal_upper) n_ru--;
    place_objects(e, &oc, n_ru, mid + 1, S - 2, 1, mid - 1);
    /* --- lower right room (custom_env.py:1880-1997) --- */
    if (!a_left && !a_upper) {
        int kx = -1, ky = -1;
        if (vl_lk) { n_rl--; place_key(e, mid + 1, S - 2, mid + 1, S - 2, gx, gy, 1, -1, -1, vl_col, vl_kib, &kx, &ky); }
        if (hr_lk) { n_rl--; place_key(e, mid + 1, S - 2, mid + 1, S - 2, gx, gy, 1, kx, ky, hr_col, hr_kib, 0, 0); }
    } else if (a_left && !a_upper) {
        if (hr_lk) { n_rl--; place_key(e, mid + 1, S - 2, mid + 1, S - 2, gx, gy, 0, -1, -1, hr_col, hr_kib, 0, 0); }
    } else if (!a_left && a_upper) {
        if (vl_lk) { n_rl--; place_key(e, mid + 1, S - 2, mid + 1, S - 2, gx, gy, 0, -1, -1, vl_col, vl_kib, 0, 0); }
    }
    if (!goal_left && !goal_upper) n_rl--;
    place_objects(e, &oc, n_rl, mid + 1, S - 2, mid + 1, S - 2);
}

static int gen_multi(env_t *e) {               /* custom_env.py:595-615 */
    static const int cmds[4] = {0, 1, 2, 5};
    int cmd = e->cfg_mission >= 0 ? e->cfg_mission : cmds[randbelow(e, 4)];
    int mid = e->S / 2;
    switch (randint(e, 2, 4)) {
        case 2: gen_2_rooms(e, mid); break;
        case 3: gen_3_rooms(e, mid); break;
        default: gen_4_rooms(e, mid); break;
    }
    return cmd;
}

/* single-room generators (custom_env.py:371-513): choice(obj_choice) on MT,
 * place_obj on PCG64 per object; [goal]; place_agent. */
static int gen_single(env_t *e) {
    static const int GTO_T[4] = {O_KEY, O_BALL, O_BOX, O_DOOR};   /* self.obj_types */
    static const int GTG_T[4] = {O_BOX, O_DOOR, O_KEY, O_BALL};
    static const int OPN_T[2] = {O_BOX, O_DOOR};
    static const int PKP_T[3] = {O_KEY, O_BOX, O_BALL};
    olist_t oc;
    int goal = 0, cmd;
    if (e->problem == P_FULL) {                 /* _generate_full_map (custom_env.py:332-369) */
        for (int t = 0; t < 4; t++)             /* for objType in obj_types: for objColor in COLOR_NAMES */
            for (int c = 0; c < 6; c++) {
                int x, y;
                place_obj(e, mk(GTO_T[t], CN2IDX[c]), &x, &y);
                add_obj(e, GTO_T[t], c, x, y);
            }
        int x, y;
        place_obj(e, mk_goal(), &x, &y);
        add_obj(e, O_GOAL, -1, x, y);
        place_agent(e);
        return rint_np(e, 0, 6);                /* np_random.choice(self.msn_commands) */
    }
    switch (e->problem) {
        case P_GTO: ol_init(&oc, GTO_T, 4); cmd = CMD_GOTO; break;
        case P_GTG: ol_init(&oc, GTG_T, 4); cmd = CMD_GOTOGOAL; goal = 1; break;
        case P_OPN: ol_init(&oc, OPN_T, 2); cmd = CMD_TOGGLE; break;
        case P_PKP: ol_init(&oc, PKP_T, 3); cmd = CMD_PICKUP; break;
        case P_DRP: ol_init(&oc, GTO_T, 4); cmd = CMD_DROP; goal = 1; break;   /* custom_env.py:515-554 */
        case P_MOV: ol_init(&oc, GTO_T, 4); cmd = CMD_MOVE; break;             /* custom_env.py:556-593 */
        default: fprintf(stderr, "oracle: unsupported problem %d\n", e->problem); abort();
    }
    if (oc.n < e->num_objects) { fprintf(stderr, "oracle: too many objects\n"); abort(); }
    for (int k = 0; k < e->num_objects; k++) {
        int t, c, x, y;
        ol_choice(e, &oc, &t, &c);
        ol_remove(&oc, t, c);
        cell_t obj = mk(t, CN2IDX[c]);
        place_obj(e, obj, &x, &y);
        add_obj(e, t, c, x, y);
    }
    if (goal) {
        int x, y;
        place_obj(e, mk_goal(), &x, &y);
        add_obj(e, O_GOAL, -1, x, y);
    }
    place_agent(e);
    return cmd;
}

static const char *type_name(int t) {
    switch (t) {
        case O_DOOR: return "door"; case O_KEY: return "key"; case O_BALL: return "ball";
        case O_BOX: return "box"; case O_GOAL: return "goal"; default: return "?";
    }
}

static void gen_grid(env_t *e) {               /* custom_env.py:122-267 */
    int S = e->S;
    for (int i = 0; i < S * S; i++) e->grid[i] = mk_none();
    e->target_action = -1; e->has_tpos = 0; e->mission[0] = 0; e->nobjs = 0;
    for (int i = 0; i < S; i++) { gset(e, i, 0, mk_wall()); gset(e, i, S - 1, mk_wall()); }
    for (int j = 0; j < S; j++) { gset(e, 0, j, mk_wall()); gset(e, S - 1, j, mk_wall()); }
    e->nrange = 0;
    int cmd = e->problem == P_MULTI ? gen_multi(e) : gen_single(e);
    /* obstacles (custom_env.py:154-172) */
    for (int k = 0; k < e->n_obstacles; k++) {
        if (e->problem == P_MULTI) {
            int mid = S / 2, x, y;
            for (;;) {
                x = randint(e, 1, S - 2);
                y = randint(e, 1, S - 2);
                if (x == mid || y == mid) continue;
                if (in_objs(e, x, y)) continue;
                if (!(x == e->ax && y == e->ay) && !next2door(e, x, y)) break;
            }
            gset(e, x, y, mk_lava());                       /* put_obj(Lava(), ...) */
        } else {
            int lava = randbelow(e, 2) == 0;                /* choice([Lava(), Wall()]) */
            int x, y;
            place_obj(e, lava ? mk_lava() : mk_wall(), &x, &y);
        }
    }
    switch (cmd) {
        case CMD_GOTO: {
            int i;
            for (;;) { i = rint_np(e, 0, e->nobjs); if (e->objs[i].type != O_GOAL) break; }
            snprintf(e->mission, sizeof e->mission, "go to %s %s", CN_NAME[e->objs[i].cname], type_name(e->objs[i].type));
            e->has_tpos = 1; e->tx = e->objs[i].x; e->ty = e->objs[i].y; e->target_action = A_DONE;
            break;
        }
        case CMD_TOGGLE: case CMD_PICKUP: {
            int i;
            for (;;) {
                i = randbelow(e, e->nobjs);
                int t = e->objs[i].type;
                if (cmd == CMD_TOGGLE && (t == O_BOX || t == O_DOOR)) break;
                if (cmd == CMD_PICKUP && (t == O_BOX || t == O_KEY || t == O_BALL)) break;
            }
            snprintf(e->mission, sizeof e->mission, "%s %s %s", CMD_NAME[cmd], CN_NAME[e->objs[i].cname], type_name(e->objs[i].type));
            e->has_tpos = 1; e->tx = e->objs[i].x; e->ty = e->objs[i].y;
            e->target_action = cmd == CMD_TOGGLE ? A_TOGGLE : A_PICKUP;
            break;
        }
        case CMD_GOTOGOAL: {
            snprintf(e->mission, sizeof e->mission, "go to goal");
            int found = 0;
            for (int i = 0; i < e->nobjs; i++)
                if (e->objs[i].type == O_GOAL) { e->has_tpos = 1; e->tx = e->objs[i].x; e->ty = e->objs[i].y; found = 1; break; }
            if (!found) { fprintf(stderr, "oracle: Invalid mission generated\n"); abort(); }
            break;
        }
        case CMD_DROP:
            snprintf(e->mission, sizeof e->mission, "drop");
            e->target_action = A_DROP;
            break;
        case CMD_MOVE: {
            static const char *DIRS[4] = {"left", "right", "up", "down"};
            int d = rint_np(e, 0, 4);                       /* np_random.choice(self.msn_directions) */
            for (int k = 1; k < S - 1; k++) {
                int x, y;
                switch (d) {
                    case 0: y = k; x = 1; while (x < S - 1 && G(e, x, y)->type != O_NONE) x++;
                        if (x < S - 1) { e->range_x[e->nrange] = x; e->range_y[e->nrange++] = y; } break;
                    case 1: y = k; x = S - 2; while (x > 0 && G(e, x, y)->type != O_NONE) x--;
                        if (x > 0) { e->range_x[e->nrange] = x; e->range_y[e->nrange++] = y; } break;
                    case 2: x = k; y = 1; while (y < S - 1 && G(e, x, y)->type != O_NONE) y++;
                        if (y < S - 1) { e->range_x[e->nrange] = x; e->range_y[e->nrange++] = y; } break;
                    default: x = k; y = S - 2; while (y > 0 && G(e, x, y)->type != O_NONE) y--;
                        if (y > 0) { e->range_x[e->nrange] = x; e->range_y[e->nrange++] = y; } break;
                }
            }
            snprintf(e->mission, sizeof e->mission, "move %s", DIRS[d]);
            break;
        }
        default: fprintf(stderr, "oracle: unsupported mission command %d\n", cmd); abort();
    }
}

/* MiniGridEnv.reset with the live-lock retry policy; returns #abandoned attempts */
static int env_reset(env_t *e, int seeded, uint64_t seed) {
    if (seeded) pcg_seed(&e->pcg, seed);
    int nll = 0;
    for (;;) {
        e->attempt_start = e->mt_words;
        e->ax = -1; e->ay = -1; e->adir = -1;
        if (setjmp(e->jb) == 0) {
            gen_grid(e);
            break;
        }
        nll++;
    }
    e->carrying = mk_none();
    e->step_count = 0;
    return nll;
}

/* ------------------------- observation (literal) ----------------------- */
static const int DV[4][2] = {{1, 0}, {0, 1}, {-1, 0}, {0, -1}};

static void gen_obs(env_t *e, uint8_t img[7][7][3]) {
    cell_t a[7][7], b[7][7];  /* [i][j] == grid(i, j) of the 7x7 view */
    int tX, tY;
    switch (e->adir) {
        case 0: tX = e->ax; tY = e->ay - 3; break;
        case 1: tX = e->ax - 3; tY = e->ay; break;
        case 2: tX = e->ax - 6; tY = e->ay - 3; break;
        default: tX = e->ax - 3; tY = e->ay - 6; break;
    }
    for (int j = 0; j < 7; j++)
        for (int i = 0; i < 7; i++) {
            int x = tX + i, y = tY + j;
            a[i][j] = (x >= 0 && x < e->S && y >= 0 && y < e->S) ? *G(e, x, y) : mk_wall();
        }
    for (int r = 0; r < e->adir + 1; r++) {       /* rotate_left: new(j, 6-i) = old(i, j) */
        for (int i = 0; i < 7; i++) for (int j = 0; j < 7; j++) b[j][6 - i] = a[i][j];
        memcpy(a, b, sizeof a);
    }
    int vis[7][7];
    for (int i = 0; i < 7; i++) for (int j = 0; j < 7; j++) vis[i][j] = e->see_through_walls;
    if (!e->see_through_walls) {                /* Grid.process_vis(agent_pos=(3, 6)) */
        vis[3][6] = 1;
        for (int j = 6; j >= 0; j--) {
            for (int i = 0; i < 6; i++) {
                if (!vis[i][j]) continue;
                if (a[i][j].type != O_NONE && !see_behind(&a[i][j])) continue;
                vis[i + 1][j] = 1;
                if (j > 0) { vis[i + 1][j - 1] = 1; vis[i][j - 1] = 1; }
            }
            for (int i = 6; i >= 1; i--) {
                if (!vis[i][j]) continue;
                if (a[i][j].type != O_NONE && !see_behind(&a[i][j])) continue;
                vis[i - 1][j] = 1;
                if (j > 0) { vis[i - 1][j - 1] = 1; vis[i][j - 1] = 1; }
            }
        }
    }
    a[3][6] = e->carrying;                      /* carrying or None */
    for (int i = 0; i < 7; i++)
        for (int j = 0; j < 7; j++) {
            if (vis[i][j]) encode_cell(&a[i][j], img[i][j]);
            else img[i][j][0] = img[i][j][1] = img[i][j][2] = 0;   /* encode(vis_mask): unseen */
        }
}

static void tokenize(const char *m, uint8_t out[32]) {   /* environment.py:91-105 */
    memset(out, 0, 32);
    for (int i = 0; m[i] && i < 32; i++) {
        char c = m[i];
        if (c >= 'A' && c <= 'Z') c = (char)(c - 'A' + 'a');
        int v;
        switch (c) {
            case ' ': v = 0; break; case '\n': v = 1; break; case '-': v = 2; break;
            case ':': v = 3; break; case ',': v = 4; break; case '.': v = 5; break;
            default: v = (c >= 'a' && c <= 'z') ? 6 + (c - 'a') : 0; break;
        }
        out[i] = (uint8_t)v;
    }
}

static double env_reward_at(env_t *e) { return 1.0 - 0.9 * ((double)e->step_count / (double)e->max_steps); }

/* PlaygroundEnv.step (custom_env.py:269-330) over MiniGridEnv.step (3P). */
static void env_step(env_t *e, int action, uint8_t img[7][7][3], double *rew, int *term, int *trunc) {
    /* --- MiniGridEnv.step --- */
    e->step_count++;
    double reward = 0.0;
    int terminated = 0, truncated = 0;
    int fx = e->ax + DV[e->adir][0], fy = e->ay + DV[e->adir][1];
    cell_t *fc = G(e, fx, fy);
    switch (action) {
        case A_LEFT: e->adir -= 1; if (e->adir < 0) e->adir += 4; break;
        case A_RIGHT: e->adir = (e->adir + 1) % 4; break;
        case A_FORWARD:
            if (fc->type == O_NONE || can_overlap(fc)) { e->ax = fx; e->ay = fy; }
            if (fc->type == O_GOAL) { terminated = 1; reward = env_reward_at(e); }
            if (fc->type == O_LAVA) terminated = 1;
            break;
        case A_PICKUP:
            if (fc->type != O_NONE && can_pickup(fc) && e->carrying.type == O_NONE) {
                e->carrying = *fc; *fc = mk_none();
            }
            break;
        case A_DROP:
            if (fc->type == O_NONE && e->carrying.type != O_NONE) { *fc = e->carrying; e->carrying = mk_none(); }
            break;
        case A_TOGGLE:
            if (fc->type == O_DOOR) {
                if (fc->is_locked) {
                    if (e->carrying.type == O_KEY && e->carrying.color == fc->color) { fc->is_locked = 0; fc->is_open = 1; }
                } else fc->is_open = !fc->is_open;
            } else if (fc->type == O_BOX) {
                *fc = fc->contains ? mk(O_KEY, fc->color) : mk_none();
            }
            break;
        case A_DONE: break;
        default: fprintf(stderr, "oracle: Unknown action %d\n", action); abort();
    }
    if (e->step_count >= e->max_steps) truncated = 1;
    gen_obs(e, img);
    /* --- PlaygroundEnv.step --- */
    int is_gtg = strcmp(e->mission, "go to goal") == 0;
    if (terminated) {
        if (!is_gtg) { e->mission_done = 0; e->has_reward = 0; reward = 0.0; }
        *rew = reward; *term = terminated; *trunc = truncated;
        return;
    }
    if (action == A_TOGGLE) {
        cell_t *f2 = G(e, e->ax + DV[e->adir][0], e->ay + DV[e->adir][1]);
        if (f2->type == O_DOOR && e->carrying.type != O_NONE && f2->color == e->carrying.color)
            e->carrying = mk_none();
    }
    int arrived = 0;
    if (!e->mission_done) {
        if (e->has_tpos) {
            if (e->target_action >= 0 && e->target_action != 0) {
                int d = e->adir;
                if ((e->ax == e->tx && e->ay - e->ty == -1 && d == 1) ||
                    (e->ax == e->tx && e->ay - e->ty == 1 && d == 3) ||
                    (e->ax - e->tx == 1 && e->ay == e->ty && d == 2) ||
                    (e->ax - e->tx == -1 && e->ay == e->ty && d == 0))
                    arrived = 1;
            } else if (e->ax == e->tx && e->ay == e->ty) {
                if (!e->has_reward) { e->reward = env_reward_at(e); e->has_reward = 1; }
                e->mission_done = 1;
            }
        }
        if (arrived && action == e->target_action) {
            if (!e->has_reward) { e->reward = env_reward_at(e); e->has_reward = 1; }
            e->mission_done = 1;
        }
        if (!e->has_tpos && action == e->target_action) {
            if (!e->has_reward) { e->reward = env_reward_at(e); e->has_reward = 1; }
            e->mission_done = 1;
        }
        for (int k = 0; k < e->nrange; k++)     /* agent_pos in target_range ('move') */
            if (e->ax == e->range_x[k] && e->ay == e->range_y[k]) {
                if (!e->has_reward) { e->reward = env_reward_at(e); e->has_reward = 1; }
                e->mission_done = 1;
                break;
            }
    }
    if (action == A_DONE) {
        if (e->mission_done) {
            e->mission_done = 0;
            double r = e->reward;   /* tmp_rew = self.reward (a float once mission_done) */
            e->has_reward = 0;
            *rew = r; *term = 1; *trunc = truncated;
            return;
        }
        if (!e->manual) {                          /* elif not self.manual (custom_env.py:325-328) */
            e->mission_done = 0; e->has_reward = 0;
            *rew = 0.0; *term = 1; *trunc = truncated;
            return;
        }
    }
    *rew = reward; *term = terminated; *trunc = truncated;
}

/* ============================ public API =============================== */
#define EXPORT __attribute__((visibility("default")))

EXPORT orc_vec *orc_create(int problem, int mission, int size, int num_objects, int all_doors_open,
                           int n_envs, int64_t base_seed, int64_t index_offset, int livelock_words,
                           int see_through_walls, int obstacles, double percent_obstacles) {
    if (size < 5 || size > MAXS || n_envs <= 0) return NULL;
    orc_vec *v = (orc_vec *)calloc(1, sizeof(orc_vec));
    v->n = n_envs;
    v->e = (env_t *)calloc((size_t)n_envs, sizeof(env_t));
    for (int i = 0; i < n_envs; i++) {
        env_t *e = &v->e[i];
        e->S = size; e->max_steps = size * size; e->problem = problem; e->cfg_mission = mission;
        e->num_objects = num_objects; e->all_doors_open = all_doors_open;
        e->see_through_walls = see_through_walls;
        /* range(floor((size - 2)**2 * percent_obstacles)) (custom_env.py:156) */
        e->n_obstacles = obstacles ? (int)floor((double)((size - 2) * (size - 2)) * percent_obstacles) : 0;
        e->livelock_words = livelock_words;
        mt_seed_int(&e->mt, (uint64_t)base_seed);          /* random.seed(c.seed), custom_env.py:82 */
        e->pcg.state = (u128)(base_seed + index_offset + i); /* overwritten at first reset */
    }
    (void)index_offset;
    return v;
}

EXPORT void orc_destroy(orc_vec *v) { if (v) { free(v->e); free(v); } }

/* PlaygroundEnv(manual=...) of every env (make_env(manual=True), environment.py:10-20). */
EXPORT void orc_set_manual(orc_vec *v, int manual) { for (int i = 0; i < v->n; i++) v->e[i].manual = manual; }

static void emit_obs(env_t *e, int i, uint8_t *img_src, uint8_t *img, uint8_t *dir, uint8_t *mis) {
    if (img) memcpy(img + (size_t)i * 147, img_src, 147);
    if (dir) dir[i] = (uint8_t)e->adir;
    if (mis) tokenize(e->mission, mis + (size_t)i * 32);
}

/* VecEnv.reset() of every env.  seeded: env i gets seed base_seed + index_offset + i
 * (SB3 VecEnv.seed / make_vec_env); unseeded: both streams continue.  The MT19937
 * stream is never re-seeded (random.seed runs once, in PlaygroundEnv.__init__). */
EXPORT void orc_reset_ex(orc_vec *v, int seeded, int64_t base_seed, int64_t index_offset,
                         uint8_t *img, uint8_t *dir, uint8_t *mis, int32_t *livelock) {
    for (int i = 0; i < v->n; i++) {
        env_t *e = &v->e[i];
        int nll = env_reset(e, seeded, (uint64_t)(base_seed + index_offset + i));
        uint8_t im[7][7][3];
        gen_obs(e, im);
        emit_obs(e, i, &im[0][0][0], img, dir, mis);
        if (livelock) livelock[i] = nll;
    }
}

EXPORT void orc_reset(orc_vec *v, int64_t base_seed, int64_t index_offset,
                      uint8_t *img, uint8_t *dir, uint8_t *mis, int32_t *livelock) {
    orc_reset_ex(v, 1, base_seed, index_offset, img, dir, mis, livelock);
}

/* One vectorised step with SubprocVecEnv auto-reset.  Outputs (NULL = skip):
 * img/dir/mis: the obs returned by env.step (the terminal obs when done);
 * r_img/r_dir/r_mis: the obs of the new episode where done; livelock: number
 * of abandoned reset attempts where done. */
EXPORT void orc_step(orc_vec *v, const int32_t *actions, uint8_t *img, uint8_t *dir, uint8_t *mis,
                     double *reward, uint8_t *term, uint8_t *trunc,
                     uint8_t *r_img, uint8_t *r_dir, uint8_t *r_mis, int32_t *livelock) {
    for (int i = 0; i < v->n; i++) {
        env_t *e = &v->e[i];
        uint8_t im[7][7][3];
        double r; int tm, tr;
        env_step(e, actions[i], im, &r, &tm, &tr);
        emit_obs(e, i, &im[0][0][0], img, dir, mis);
        if (reward) reward[i] = r;
        if (term) term[i] = (uint8_t)tm;
        if (trunc) trunc[i] = (uint8_t)tr;
        if (livelock) livelock[i] = 0;
        if (tm || tr) {
            int nll = env_reset(e, 0, 0);
            gen_obs(e, im);
            emit_obs(e, i, &im[0][0][0], r_img, r_dir, r_mis);
            if (livelock) livelock[i] = nll;
        }
    }
}

/* CPU baseline leg of bench.py (cpu_baseline): `steps` vectorised steps of every env with
 * uniform random actions on 0..6 (xorshift64*, seeded), auto-reset included, each step's
 * observation emitted (image HWC, direction, mission tokens) into scratch -- the work of
 * PlaygroundEnv.step + gen_obs + the two wrappers per env-step, without Python overhead.
 * Returns the number of auto-resets. */
uint8_t orc_bench_sink[147 + 1 + 32];      /* emitted obs land here (global: not dead stores) */
EXPORT int64_t orc_bench(orc_vec *v, int64_t steps, uint64_t seed) {
    uint64_t x = seed * 0x9E3779B97F4A7C15ULL + 1;
    uint8_t *img = orc_bench_sink, *dir = orc_bench_sink + 147, *mis = orc_bench_sink + 148;
    int64_t resets = 0;
    for (int64_t t = 0; t < steps; t++) {
        for (int i = 0; i < v->n; i++) {
            env_t *e = &v->e[i];
            x ^= x >> 12; x ^= x << 25; x ^= x >> 27;
            const int a = (int)(((x * 0x2545F4914F6CDD1DULL) >> 32) % 7u);
            uint8_t im[7][7][3];
            double r; int tm, tr;
            env_step(e, a, im, &r, &tm, &tr);
            emit_obs(e, 0, &im[0][0][0], img, dir, mis);
            if (tm || tr) {
                env_reset(e, 0, 0);
                gen_obs(e, im);
                emit_obs(e, 0, &im[0][0][0], img, dir, mis);
                resets++;
            }
        }
    }
    return resets;
}

/* State dump in the fixture layout (tests/golden/make_golden.py). */
EXPORT void orc_dump(orc_vec *v, uint8_t *grid /*[n][S][S][4] x-major*/, uint8_t *agent /*[n][3]*/,
                     uint8_t *carrying /*[n][4]*/, int32_t *step_count, uint8_t *mission_done,
                     double *stored_reward, int64_t *mtwords, uint64_t *pcg /*[n][6]*/,
                     uint8_t *target /*[n][3]*/) {
    for (int i = 0; i < v->n; i++) {
        env_t *e = &v->e[i];
        int S = e->S;
        if (grid)
            for (int x = 0; x < S; x++)
                for (int y = 0; y < S; y++) {
                    uint8_t *o = grid + (((size_t)i * S + x) * S + y) * 4;
                    encode_cell(G(e, x, y), o);
                    o[3] = (G(e, x, y)->type == O_BOX && G(e, x, y)->contains) ? 1 : 0;
                }
        if (agent) { agent[i * 3] = (uint8_t)e->ax; agent[i * 3 + 1] = (uint8_t)e->ay; agent[i * 3 + 2] = (uint8_t)e->adir; }
        if (carrying) {
            uint8_t *o = carrying + i * 4;
            if (e->carrying.type == O_NONE) { o[0] = o[1] = o[2] = o[3] = 0; }
            else { encode_cell(&e->carrying, o); o[3] = (e->carrying.type == O_BOX && e->carrying.contains) ? 1 : 0; }
        }
        if (step_count) step_count[i] = e->step_count;
        if (mission_done) mission_done[i] = (uint8_t)e->mission_done;
        if (stored_reward) stored_reward[i] = e->has_reward ? e->reward : NAN;
        if (mtwords) mtwords[i] = e->mt_words;
        if (pcg) {
            uint64_t *o = pcg + i * 6;
            o[0] = (uint64_t)(e->pcg.state >> 64); o[1] = (uint64_t)e->pcg.state;
            o[2] = (uint64_t)(e->pcg.inc >> 64); o[3] = (uint64_t)e->pcg.inc;
            o[4] = (uint64_t)e->pcg.has_uint32; o[5] = e->pcg.uinteger;
        }
        if (target) {
            target[i * 3] = e->has_tpos ? (uint8_t)e->tx : 255;
            target[i * 3 + 1] = e->has_tpos ? (uint8_t)e->ty : 255;
            target[i * 3 + 2] = e->target_action < 0 ? 255 : (uint8_t)e->target_action;
        }
    }
}

/* Mission string of env i (for tests). */
EXPORT const char *orc_mission(orc_vec *v, int i) { return v->e[i].mission; }

/* ---- RNG known-answer hooks (pinned against CPython / numpy in tests) --- */
EXPORT void orc_mt_words(uint64_t seed, int n, uint32_t *out) {
    mt_t m; mt_seed_int(&m, seed);
    for (int i = 0; i < n; i++) out[i] = mt_next(&m);
}
EXPORT void orc_pcg_seed_state(uint64_t seed, uint64_t out[4]) {
    pcg_t p; pcg_seed(&p, seed);
    out[0] = (uint64_t)(p.state >> 64); out[1] = (uint64_t)p.state;
    out[2] = (uint64_t)(p.inc >> 64); out[3] = (uint64_t)p.inc;
}
EXPORT void orc_pcg_integers(uint64_t seed, int n, const int64_t *lo, const int64_t *hi, int64_t *out) {
    pcg_t p; pcg_seed(&p, seed);
    for (int i = 0; i < n; i++) out[i] = pcg_integers(&p, lo[i], hi[i]);
}
