"""Host model of the refill's production policy (refill_body + the slide's round cap), to see which policy keeps
the lanes' ring levels off the 2K floor over long runs (DESIGN §5 steady state).  Per 20-step epoch each env pops
Binomial(20, 1/7) episodes (the 'done' action ends an episode with probability 1/7 per step under uniform random
actions; a rare max_steps end ignored), every attempt is abandoned with probability 0.9 % (the measured rate), and
a wave's rounds are its busiest lane's.  Policies: 'product' (cap = min(ceil(wave mean consumption), round cap));
'global' (cap = the round cap for every lane).  Prints the mean level, the lanes below 2K and the mean / max rounds
per wave over time."""
import numpy as np

def run(policy, epochs=1000, n=65536, D=256, K=20, seed=0, margin=9.0):
    rng = np.random.default_rng(seed)
    lv = np.full(n, D, dtype=np.int64)
    acc = 0
    cons_last = np.zeros(n, dtype=np.int64)
    out = []
    for ep in range(epochs):
        mean = cons_last.mean() if ep else 2.9
        tgt = mean * (1 + margin / (D - 2 * K))
        acc1 = acc + int(tgt * 1024 + 0.5)
        rc = max((acc1 >> 10) - (acc >> 10), 1)
        acc = acc1
        space = D - lv
        need = np.maximum(2 * K - lv, 0)
        if policy == "product":
            wm = np.ceil(cons_last.reshape(-1, 64).mean(1) if ep else np.full(n // 64, 3.0)).astype(np.int64)
            cap = np.minimum(np.repeat(wm, 64), rc)
        else:
            cap = np.full(n, rc)
        nfree = np.minimum(np.maximum(need, np.minimum(cap, space)), space)
        # attempts: each attempt succeeds w.p. 0.991; an abandoned one costs a unit unless the lane is at need
        att = nfree.copy()
        ab = rng.binomial(att, 0.009)
        prod = nfree - np.where(nfree > need, np.minimum(ab, nfree - need), 0)
        extra_rounds = np.where(need > 0, ab, 0)            # a lane at need retries within the epoch
        rounds = (nfree + extra_rounds).reshape(-1, 64).max(1)
        c = rng.binomial(K, 1.0 / 7.0, n)
        lv = lv + prod - c
        cons_last = c
        if ep % 100 == 99:
            out.append((ep + 1, round(float(lv.mean()), 1), int((lv < 2 * K).sum()), round(float(rounds.mean()), 2), int(rounds.max())))
    return out

if __name__ == "__main__":
    for pol in ("product", "global"):
        print(pol, run(pol))
