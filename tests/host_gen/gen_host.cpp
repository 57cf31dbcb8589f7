// gen_host.cpp -- TEST INFRASTRUCTURE: the engine's episode generator (minigrid-rl_amd/csrc/mgx_device.h,
// reset_env) compiled for the host, one env after the other, so that a change to its draw order can be
// checked against the C oracle (oracle/mgx_oracle.c) on CPU in seconds (tests/test_generator_host.py).
// The GPU parity tests (-m gpu) remain the proof; this is the generator alone, not the kernels around it.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "mgx_device.h"

using namespace mgx;

namespace {
struct MT {                                         // CPython random.seed(n) + genrand_uint32
    uint32_t mt[624];
    int mti;
    void init(uint32_t s) {
        mt[0] = s;
        for (int i = 1; i < 624; i++) mt[i] = 1812433253U * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
        mti = 624;
    }
    void seed(uint64_t n) {
        uint32_t key[2];
        int klen = 0;
        if (n == 0) key[klen++] = 0;
        while (n) { key[klen++] = (uint32_t)n; n >>= 32; }
        init(19650218U);
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

template <int NW, bool EXT>
int run(int problem, int mission, int S, int nobj, int ado, int n_obst, int n, int64_t seed, int episodes,
        const std::vector<uint64_t> &tab, uint8_t *grids, uint8_t *agent, uint8_t *target, int64_t *cursor,
        uint64_t *pcg, int32_t *livelock) {
    constexpr int WS = win_stride<NW>();
    std::vector<uint32_t> win(WS + 2), objs(MAX_OBJS + 1);
    std::vector<uint8_t> g((size_t)S * S + 16);
    uint32_t err = 0;
    for (int i = 0; i < n; i++) {
        Gen<NW> G;
        G.g = g.data();
        G.S = S;
        G.table = tab.data();
        G.rmask = (uint64_t)tab.size() - MT_PAD - 1;      // the table is one unwrapped ring (power of two)
        G.tlo = 0;
        G.thi = G.rmask + 1;
        G.win = reinterpret_cast<uint64_t *>(win.data());
        G.objs = objs.data();
        G.llw = 4096;
        G.err = 0;
        G.problem = problem; G.cfg_mission = mission; G.num_objects = nobj; G.all_doors_open = ado;
        G.n_obstacles = n_obst;
        G.abort = false; G.nobjs = 0; G.ax = G.ay = -1; G.adir = 0;
        G.phave = false; G.prec = 0;                       // no prefix records on the host: every prefix drawn
        gen_init(G);
        pcg_seed(G.pcg, (uint64_t)(seed + i));
        G.cur = 0;
        G.gbase = ~0ull >> 1;
        for (int k = 0; k < episodes; k++) {
            ResetOut R;
            reset_env<NW, EXT>(G, R);
            const size_t o = (size_t)i * episodes + k;
            std::memcpy(grids + o * S * S, G.g, (size_t)S * S);
            agent[o * 3] = (uint8_t)G.ax; agent[o * 3 + 1] = (uint8_t)G.ay; agent[o * 3 + 2] = (uint8_t)G.adir;
            target[o * 4] = R.tx; target[o * 4 + 1] = R.ty; target[o * 4 + 2] = R.ta; target[o * 4 + 3] = R.mission_id;
            cursor[o] = (int64_t)G.cur;
            pcg[o * 4] = G.pcg.sh; pcg[o * 4 + 1] = G.pcg.sl; pcg[o * 4 + 2] = G.pcg.has; pcg[o * 4 + 3] = G.pcg.uinteger;
            livelock[o] = R.livelocks;
        }
        err |= G.err;
    }
    return (int)err;
}
}  // namespace

extern "C" int hg_run(int problem, int mission, int S, int nobj, int ado, int n_obst, int n, int64_t seed,
                      int episodes, uint8_t *grids, uint8_t *agent, uint8_t *target, int64_t *cursor, uint64_t *pcg,
                      int32_t *livelock) {
    // the packed MT19937(seed) stream (mgx_create's table: ten top-5-bit fields per group) + the mirror pad
    const int64_t groups = 1 << 18;
    std::vector<uint64_t> tab((size_t)groups + MT_PAD, 0ull);
    MT m;
    m.seed((uint64_t)seed);
    for (int64_t w = 0; w < groups * MT_FIELDS; w++) {
        const uint64_t f = m.next() >> 27;
        tab[(size_t)(w / MT_FIELDS)] |= f << (6 * (w % MT_FIELDS));
    }
    for (int k = 0; k < MT_PAD; k++) tab[(size_t)groups + k] = tab[(size_t)k];
    const int nw = S * S <= 64 ? 1 : (S * S <= 128 ? 2 : 4);
    const bool ext = n_obst > 0 || problem == 1 || problem == 6 || problem == 7;
#define HG(NW_, EXT_) return run<NW_, EXT_>(problem, mission, S, nobj, ado, n_obst, n, seed, episodes, tab, grids, agent, target, cursor, pcg, livelock)
    if (!ext) { if (nw == 1) HG(1, false); if (nw == 2) HG(2, false); HG(4, false); }
    if (nw == 1) HG(1, true);
    if (nw == 2) HG(2, true);
    HG(4, true);
#undef HG
}
