"""How far FMA contraction alone moves the reference-order fluxes (CPU, oracle only -- test tooling).

The reference was built by g++-14 -O3 -std=gnu++11 on arm64 (/root/reference/setup.py:7-8, 27): GCC contracts a*b+c
into fused multiply-adds there by default, and its GSL / libm are Homebrew's and Apple's.  The oracle (and the GPU,
bit for bit) evaluates every expression uncontracted (-ffp-contract=off).  This script evaluates every point of a
config three times in the reference order (GSL's algorithms, oracle.reference_order(1)):

* base   -- oracle/_build/libnusi_oracle.so (-ffp-contract=off; the parity oracle);
* fc     -- oracle/_build/libnusi_oracle_fc.so: the restated reference code and GSL at -O3 -ffp-contract=fast (GCC's
            contraction of the reference's own expressions), the libm stand-in unchanged;
* fcall  -- oracle/_build/libnusi_oracle_fcall.so: every file contracted, the libm stand-in included;

and records the max relative flux difference of fc / fcall against base per config.  That spread is a floor below
which parity with the reference's own binary is unpinned: two equally valid IEEE evaluations of the same algorithm
differ by it.  It is not a tolerance of this implementation (which is <= 1e-11 of base).

  make -C oracle fc && python scripts/contraction_floor.py [c1 c2a c2b c4 c3] > profiles/r6/contraction_floor.json
"""
import concurrent.futures as cf
import json
import multiprocessing as mp
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VARIANTS = {"base": "libnusi_oracle.so", "fc": "libnusi_oracle_fc.so", "fcall": "libnusi_oracle_fcall.so"}
_PP = None


def _init(variant, pp):
    """Worker initialiser: select the oracle build before oracle.py is first imported in this process."""
    global _PP
    os.environ["NUSI_ORACLE_LIB"] = os.path.join(ROOT, "oracle", "_build", VARIANTS[variant])
    _PP = pp


def _evolve(kw):
    from oracle import oracle
    o = oracle.Oracle(**kw)
    if _PP is not None:
        o.load_phiphi(*_PP)
    with oracle.reference_order(1):
        return o.evolve()[1]


def run_variant(variant, pts, pp=None, procs=None):
    import numpy as np
    procs = procs or int(os.environ.get("NPROC", "8"))
    with cf.ProcessPoolExecutor(min(procs, len(pts)), mp_context=mp.get_context("spawn"), initializer=_init,
                                initargs=(variant, pp)) as ex:
        return np.stack(list(ex.map(_evolve, pts, chunksize=max(1, len(pts) // (4 * procs)))))


def configs(names, pp_dir=None):
    from tests import cases
    out = {}
    for name in names:
        if name == "c1":
            out[name] = ([dict(cases.TEST_CPP, N_bins_E=300)], None)
        elif name == "c2a":
            out[name] = ([cases.C2A], None)
        elif name == "c2b":
            out[name] = ([cases.C2B], None)
        elif name == "c4":
            out[name] = (cases.scan_points(), None)
        elif name == "c3":
            from nusiprop_amd.phiphi_tables import write_synthetic_tables
            from tests.test_phiphi import C3
            at, atd, a, ad = write_synthetic_tables(pp_dir or "/tmp/nusi_pp_ref")
            out[name] = ([C3], (at, atd, a, ad))
    return out


def main():
    import numpy as np
    from tests import cases
    names = sys.argv[1:] or ["c1", "c2a", "c2b", "c4", "c3"]
    res = {"what": "max relative flavour-flux difference of the contracted oracle builds against the parity oracle "
                   "(-ffp-contract=off), all in the reference order (GSL's algorithms); a floor below which parity "
                   "with the reference's own binary (g++ -O3 on arm64, FMA contraction, Apple libm) is unpinned",
           "variants": {"fc": "reference code + GSL restatement at -O3 -ffp-contract=fast, libm stand-in uncontracted",
                        "fcall": "every oracle file at -O3 -ffp-contract=fast (libm stand-in too)"},
           "script": "scripts/contraction_floor.py", "configs": {}}
    for name, (pts, pp) in configs(names).items():
        kws = [cases.oracle_kwargs(p) for p in pts]
        fl = {v: run_variant(v, kws, pp) for v in VARIANTS}
        rec = {"points": len(pts)}
        for v in ("fc", "fcall"):
            d = np.array([cases.rel_err(fl[v][k], fl["base"][k]) for k in range(len(pts))])
            r = {"max": float(d.max()), "median": float(np.median(d)), "points_above_1e-11": int(np.sum(d > 1e-11)),
                 "points_above_1e-9": int(np.sum(d > 1e-9))}
            if len(pts) > 1:
                w = np.argsort(-d)[:8]
                r["worst"] = [dict(index=int(i), mphi=pts[i]["mphi"], g=pts[i]["g"], rel=float(d[i])) for i in w]
            rec[v] = r
        res["configs"][name] = rec
        print("%s: fc max %.3g, fcall max %.3g" % (name, rec["fc"]["max"], rec["fcall"]["max"]), file=sys.stderr)
    json.dump(res, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
