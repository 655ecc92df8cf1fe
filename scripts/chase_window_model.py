"""How much a windowed miss chase could save, on the slot-form model.

The encoder's miss chase (hc_fgk.hip: Fgk::chase) climbs from a leaf one parent per LDS round
trip (~13 instructions a level). The windowed variant would read the 64 weight words above the
current position at once (one lane-parallel round trip) and follow the parent fields inside that
window by lane reads (~5 instructions a level); a parent past the window opens a new one.

For each miss of the path cache (tests/fgk_cache_model.py: PathCache, the kernel's insert depth
and probe after 7 levels) this counts the levels the chase climbs and how many of them a
64-position window starting at the climb's current position would serve.

    python scripts/chase_window_model.py [--streams 2] [--symbols 60000]
"""
import argparse
import os
import sys

ROOT_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT_DIR, "oracle"))
sys.path.insert(0, os.path.join(ROOT_DIR, "tests"))

import numpy as np  # noqa: E402
import oracle  # noqa: E402
from fgk_cache_model import ROOT, MAXD, PathCache, Tree  # noqa: E402

INSERT_DEPTH = 9  # hc_fgk.hip HC_INSERT_DEPTH
PROBE = 7         # hc_fgk.hip HC_PROBE
WINDOW = 64


def chase_levels(t, pc, x):
    """the positions the kernel's chase climbs through for a miss at leaf x (before the probe's
    cached row supplies the rest, or up to the root)"""
    climbed, c, d = [], x, 0
    while c != ROOT:
        climbed.append(c)
        c = t.up[c]
        d += 1
        if d == PROBE:
            for e in range(len(pc.ent)):
                if pc.ent[e] is not None and c in pc.ent[e][1]:
                    return climbed
    return climbed


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--symbols", type=int, default=60000)
    a = ap.parse_args()
    misses = levels = windows = in_window = 0
    dist = []
    for k in range(a.streams):
        syms = np.frombuffer(oracle.rle(oracle.diff(oracle.synth("photo", k))), np.uint8)[: a.symbols]
        t, pc = Tree(), PathCache()
        for sym in syms.tolist():
            if t.where[sym] == 0:
                t.split(sym)
            x = t.where[sym]
            if pc.lookup(sym) is None:
                pv = t.path(x)
                misses += 1
                cl = chase_levels(t, pc, x)
                levels += len(cl)
                base = None
                for c in cl:
                    p = t.up[c]
                    dist.append(p - c)
                    if base is None or c - base >= WINDOW:  # c itself must be in the window
                        base = c
                        windows += 1
                    if p - base < WINDOW:
                        in_window += 1
                if len(pv) <= INSERT_DEPTH and len(pv) <= MAXD:
                    pc.insert(sym, pv)
            t.update(x)
            for s, lead in t.swaps:
                pc.on_swap(s, lead)
    d = np.array(dist)
    print(f"streams {a.streams} x {a.symbols} photo -c -m symbols: misses {misses}, chased levels {levels} "
          f"({levels / max(misses, 1):.2f} per miss)")
    print(f"parent distance per chased level: median {np.median(d):.0f}, <64: {np.mean(d < 64) * 100:.1f} %, "
          f"<16: {np.mean(d < 16) * 100:.1f} %")
    print(f"64-wide windows: {windows} window reads for {levels} levels ({windows / max(levels, 1):.2f} per level), "
          f"levels whose parent is inside the current window: {in_window / max(levels, 1) * 100:.1f} %")
    # issue slots from the gfx950 ISA of the two builds (hc_fgk.hip chase, HC_CHASE_WIN 0 / 1):
    # a chased level = DPP shift, select, address, LDS read, mask, readfirstlane, compare, branch
    # (~9); a windowed level = window test (sub, compare, branch), DPP shift, move, select, lane
    # read, root compare, branch (~9) plus ~8 for each window read
    now = 9 * levels
    win = 8 * windows + 9 * levels
    print(f"instructions (estimate): chase {now / max(misses, 1):.1f} per miss, windowed {win / max(misses, 1):.1f}; "
          f"round trips per miss {levels / max(misses, 1):.2f} -> {windows / max(misses, 1):.2f}")


if __name__ == "__main__":
    main()
