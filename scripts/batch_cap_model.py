"""How often the FGK batches stop at their lane cap, and what a second lane layout would buy
(DESIGN.md §8 item 1), on the slot-form model (tests/fgk_batch_model.py, fgk_cache_model.py).

Both kernels batch seven symbols per step, nine lanes each (lane 9 j + l: level l of symbol j's
path; levels 0..8). A step ends at the first symbol that fails the tentative leader test, has no
cached path (encoder) / no leaf in the level tables (decoder), or at the cap. The alternative
counted here: ten symbols of six lanes (depth <= 5) whenever the step's next ten symbols all fit
that depth, else the present layout.

    python scripts/batch_cap_model.py [--stream 0] [--symbols 60000]
"""
import argparse
import os
import sys

ROOT_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT_DIR, "oracle"))
sys.path.insert(0, os.path.join(ROOT_DIR, "tests"))

import numpy as np  # noqa: E402
import oracle  # noqa: E402
import fgk_batch_model as M  # noqa: E402
from fgk_cache_model import ROOT, PathCache, Tree  # noqa: E402


def run(symbols, encoder, layout):
    """layout(path_of, symbols, i) -> (cap, deepest path length); path_of(sym, depth) is the
    symbol's batch path (ROOT last) or None"""
    t, pc = Tree(), PathCache()
    st = {"steps": 0, "alone": 0, "full": 0}

    def alone(sym):
        if t.where[sym] == 0:
            t.split(sym)
        x = t.where[sym]
        if encoder and pc.lookup(sym) is None:
            pc.insert(sym, t.path(x))
        t.update(x)
        for s, lead in t.swaps:
            pc.on_swap(s, lead)

    def path_of(sym, depth):
        if t.where[sym] == 0:
            return None
        if encoder:
            e = pc.slot.get(sym)
            p = pc.ent[e][1] if e is not None else None
        else:
            p = t.path(t.where[sym])
        return p + [ROOT] if p is not None and len(p) <= depth else None

    i, n = 0, len(symbols)
    while i < n:
        cap, depth = layout(path_of, symbols, i)
        paths = []
        for s in symbols[i:i + cap]:
            paths.append(path_of(s, depth))
            if paths[-1] is None:
                break
        jf = M.tentative_len(t, paths)
        st["steps"] += 1
        st["full"] += jf == cap
        for p in paths[:jf]:
            for a in p:
                t.w[a] += 1
        i += jf
        if jf < len(paths) and i < n:
            st["alone"] += 1
            alone(symbols[i])
            i += 1
    return st


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stream", type=int, default=0)
    ap.add_argument("--symbols", type=int, default=60000)
    a = ap.parse_args()
    syms = np.frombuffer(oracle.rle(oracle.diff(oracle.synth("photo", a.stream))), np.uint8)[: a.symbols].tolist()
    for name, enc in (("encoder (path cache)", True), ("decoder (level tables)", False)):
        # the deepest batch path: the encoder's cached rows (insert depth 9), the decoder's tables
        # (codes of up to 8 bits)
        deep = 9 if enc else 8
        now = lambda path_of, s, i, deep=deep: (7, deep)  # noqa: E731

        def hybrid(path_of, s, i, deep=deep):
            return (10, 5) if all(path_of(x, 5) is not None for x in s[i:i + 10]) else (7, deep)

        a0, a1 = run(syms, enc, now), run(syms, enc, hybrid)
        print(f"{name}: 7 x 9 lanes: {a0['steps']} steps, {a0['full'] / a0['steps'] * 100:.0f} % full, "
              f"{len(syms) / a0['steps']:.2f} symbols a step, {a0['alone']} alone; "
              f"+ 10 x 6 when the next ten fit: {a1['steps']} steps ({(a1['steps'] / a0['steps'] - 1) * 100:+.1f} %), "
              f"{len(syms) / a1['steps']:.2f} a step, {a1['alone']} alone")


if __name__ == "__main__":
    main()
