"""CPU model of the piece screen's candidate load: builds the panel's piece
table as build_pieces (csrc/dmx_api.cpp) does, then counts per read the sampled 8-mer lookups,
bitmap hits (candidates), entries checked and verified copies, and the per-(part, 64-position
step) candidate counts that set the screen's wave divergence.

Usage: python tools/piece_sim.py [config] [n_reads] [round]   (round 0: SP5 FRONT, 1: SP27 BACK)
"""
import os
import sys
from collections import defaultdict

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "nanopore-barcoding-orc_amd"))
from dmx import synth  # noqa: E402

CODE = {"A": 0, "C": 1, "G": 2, "T": 3}


def acc_full(m, e=0.1):
    return int(m * e + 1e-12)


def build(panel, n_orient=2, e=0.1):
    pcs = []
    for s in panel:
        m = len(s)
        K = acc_full(m, e)
        np_ = K + 1
        for p in range(np_):
            r0, r1 = p * m // np_, (p + 1) * m // np_
            ln = min(16, r1 - r0)
            re = r0 + ln
            for o in range(n_orient):
                v = 0
                for i in range(ln):
                    cd = CODE[s[r0 + i]] if o == 0 else 3 - CODE[s[re - 1 - i]]
                    v |= cd << (2 * i)
                pcs.append((v, ln, o, (m - re) - K, (m - re) + K))
    uq = {}
    for v, ln, o, dlo, dhi in pcs:
        k = (v, ln, o)
        if k in uq:
            uq[k] = (min(uq[k][0], dlo), max(uq[k][1], dhi))
        else:
            uq[k] = (dlo, dhi)
    minlen = min(k[1] for k in uq)
    step = 4 if minlen - 7 >= 4 else (2 if minlen - 7 >= 2 else 1)
    mult = defaultdict(int)
    for (v, ln, o) in uq:
        for off in range(ln - 8 + 1):
            mult[(v >> (2 * off)) & 0xFFFF] += 1
    ents = defaultdict(list)
    for (v, ln, o), (dlo, dhi) in uq.items():
        best, bc = 0, 1 << 30
        for j0 in range(ln - 8 - step + 2):
            c = sum(mult[(v >> (2 * off)) & 0xFFFF] for off in range(j0, j0 + step))
            if c < bc:
                bc, best = c, j0
        for off in range(best, best + step):
            ents[(v >> (2 * off)) & 0xFFFF].append((v, ln, o, off, dlo, dhi))
    return ents, step, len(uq)


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2x24"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    rnd = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    d = synth.generate(cfg, n=n)
    panel = d["sp5"] if rnd == 0 else d["sp27"]
    ents, step, npieces = build(panel)
    nkeys = len(ents)
    print(f"pieces {npieces} keys {nkeys} entries {sum(len(v) for v in ents.values())} step {step}"
          f" key density {nkeys / 65536:.4f}")
    mult = sorted((len(v) for v in ents.values()), reverse=True)
    print("largest key lists", mult[:10])
    looks = cands = checks = hits = 0
    step_c = []
    for s in synth.to_strings(d):
        codes = [CODE.get(c, 0) for c in s]
        L = len(codes)
        kv = 0
        kms = [0] * max(0, L - 7)
        for i, c in enumerate(codes):
            kv = ((kv >> 2) | (c << 14)) & 0xFFFF
            if i >= 7:
                kms[i - 7] = kv
        per_step = defaultdict(int)
        for x in range(0, max(0, L - 7), step):
            looks += 1
            lst = ents.get(kms[x])
            if lst:
                cands += 1
                per_step[x // 64] += 1
                checks += len(lst)
                for v, ln, o, off, dlo, dhi in lst:
                    g = x - off
                    if g < 0 or g + ln > L:
                        continue
                    w = 0
                    for i in range(ln):
                        w |= codes[g + i] << (2 * i)
                    hits += w == v
        step_c += [per_step.get(k, 0) for k in range((L + 63) // 64)]
    sc = np.array(step_c)
    print(f"reads {n}: lookups/read {looks / n:.1f} candidates/read {cands / n:.2f} "
          f"entries checked/read {checks / n:.2f} verified copies/read {hits / n:.2f}")
    print(f"per 64-position step: mean candidates {sc.mean():.3f}, P(>=1) {(sc >= 1).mean():.3f}, "
          f"P(>=2) {(sc >= 2).mean():.3f}, max {sc.max()}")
    # expected wave iterations: max over 64 random lane-steps
    rng = np.random.default_rng(0)
    sims = rng.choice(sc, size=(20000, 64)).max(axis=1)
    print(f"E[max over a wave's 64 lane-steps] {sims.mean():.2f}")


if __name__ == "__main__":
    main()
