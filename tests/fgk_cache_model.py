"""Python model of the FGK kernels' two caches (hc_fgk.hip), checked against the plain slot form.

The slot-form tree (oracle/hc_oracle.c: sl_*) changes shape only at a split
(new leaves below the NYT position) and at a swap (the contents of positions s and lead trade
places, huffman.cpp:186-217). Two caches exploit that:

* path cache (encoder): the root paths (positions, code bits) of up to 16 recently coded
  symbols whose paths are at most 12 deep; a new path takes an entry dropped by a swap (or
  never used) first, else the FIFO hand's. A swap of s and lead stales exactly the cached paths that contain s or
  lead; a split stales none (the NYT position is on no symbol's path).
* level tables (decoder): for j = 1..8 and each j-bit prefix, the position reached from the root
  by reading the prefix's bits (stopping at a leaf). The 8-bit table finds the leaf; lane 64-j
  reads level j's entry for the prefix, so the whole root path arrives in one lane-parallel
  read. They go stale only when a swap moves the content of an inner position that some walk
  passes THROUGH (marked at build time); positions where a walk ENDS are read again at lookup
  time, so a swap or split there costs at most a longer (continued) descent.

`run(symbols)` codes the stream with both caches, asserts at every symbol that a cache hit equals
a fresh chase and that a table lookup equals a full descent, and returns hit / rebuild counts.
"""

ROOT = 512
INNER = 0x100
NYT = 0x200
SLOTS = 16
MAXD = 12  # deepest cached path
REFRESH = 16  # rebuild the level tables after this many lookups they left short


class Tree:
    def __init__(self):
        self.w = [0] * 514
        self.w[513] = 1 << 62
        self.up = [0] * 513
        self.body = [0] * 513
        self.body[ROOT] = NYT
        self.where = [0] * 256
        self.nyt = ROOT
        self.swaps = []  # (s, lead) of the current update

    def relink(self, b, pos):
        if b & INNER:
            c = (b & 255) * 2
            self.up[c] = self.up[c + 1] = pos
        elif not b & NYT:
            self.where[b] = pos

    def split(self, s):
        z = self.nyt
        self.body[z] = INNER | ((z - 2) >> 1)
        self.body[z - 2] = NYT
        self.body[z - 1] = s
        self.w[z - 2] = self.w[z - 1] = 0
        self.up[z - 2] = self.up[z - 1] = z
        self.where[s] = z - 1
        self.nyt = z - 2

    def update(self, x):
        self.swaps = []
        while x != ROOT:
            f = self.w[x]
            lead = x
            while self.w[lead + 1] == f:
                lead += 1
            if lead != x and lead != self.up[x]:
                a, c = self.body[x], self.body[lead]
                self.body[x], self.body[lead] = c, a
                self.relink(c, x)
                self.relink(a, lead)
                self.swaps.append((x, lead))
                x = lead
            self.w[x] += 1
            x = self.up[x]
        self.w[ROOT] += 1

    def path(self, x):
        pv = []
        while x != ROOT:
            pv.append(x)
            x = self.up[x]
        return pv  # level 0 = the leaf; code bits = [p & 1 for p in reversed(pv)]

    def descend(self, bits, i):
        x, d = ROOT, 0
        while self.body[x] & INNER:
            x = (self.body[x] & 255) * 2 + bits[i + d]
            d += 1
        return x, d


class PathCache:
    """As the kernel: an insert takes the lowest-numbered free entry (dropped by a swap, or
    never used), else the entry at the FIFO hand `next`; a hit changes nothing."""

    def __init__(self):
        self.ent = [None] * SLOTS  # (sym, pv)
        self.slot = {}             # sym -> slot
        self.next = 0
        self.hits = self.misses = self.inval = self.probes = 0

    def lookup(self, sym):
        e = self.slot.get(sym)
        if e is None:
            self.misses += 1
            return None
        self.hits += 1
        return self.ent[e][1]

    def insert(self, sym, pv):
        if len(pv) > MAXD:
            return
        # an entry dropped by a swap (or never used) first, lowest number; otherwise FIFO
        free = [e for e in range(SLOTS) if self.ent[e] is None]
        if free:
            e = free[0]
        else:
            e = self.next
            self.next = (e + 1) % SLOTS
        if self.ent[e] is not None:
            self.slot.pop(self.ent[e][0], None)
        self.ent[e] = (sym, list(pv))
        self.slot[sym] = e

    def probe(self, t, x, levels=7):
        """The encoder's miss chase (hc_fgk.hip: chase + pc_probe): climb `levels` levels from
        x, then take the rest of the root path from the first entry (lowest number, then lowest
        level) whose path holds the position reached. None: the climb reached the root or no
        entry holds it (the kernel then chases on)."""
        up, c = [], x
        for _ in range(levels):
            up.append(c)
            c = t.up[c]
            if c == ROOT:
                return None
        for e in range(SLOTS):
            if self.ent[e] is not None and c in self.ent[e][1]:
                row = self.ent[e][1]
                return up + row[row.index(c):]
        return None

    def on_swap(self, s, lead):
        for e in range(SLOTS):
            if self.ent[e] is not None and (s in self.ent[e][1] or lead in self.ent[e][1]):
                self.slot.pop(self.ent[e][0], None)
                self.ent[e] = None
                self.inval += 1


class LevelTables:
    """L_j[p] for j = 1..8 and every j-bit prefix p: (position, depth) where the walk from the root
    along p's bits stops (a leaf above depth j keeps its entry). Built breadth first, one level
    at a time, as the kernel does; `through` = inner positions some walk passes (depth < 8): the
    kernel's generation marks, which a partial rebuild adds to and only a full one clears."""

    def __init__(self):
        self.L = {0: [(ROOT, 0)]}
        self.through = set()
        self.frm = 0  # rebuild levels frm..8 (9: none, 0: all)
        self.short = 0
        self.rebuilds = self.cont = 0

    def build(self, t):
        j0 = self.frm
        if j0 == 0:
            self.through = set()
            self.short = 0
            j0 = 1
        prev = self.L[j0 - 1]
        for j in range(j0, 9):
            cur = []
            for q in range(1 << j):
                x, dep = prev[q >> 1]
                if dep == j - 1 and t.body[x] & INNER:
                    self.through.add(x)
                    cur.append(((t.body[x] & 255) * 2 + (q & 1), j))
                else:
                    cur.append((x, dep))
            self.L[j] = cur
            prev = cur
        self.frm = 9
        self.rebuilds += 1

    def table_level(self, s, lead):
        """the shallowest level < 8 holding position s or lead (8: none), scanning entries in
        index order as the kernel's table_level does"""
        for j in range(1, 8):
            if any(x in (s, lead) for x, _ in self.L[j]):
                return j
        return 8

    def on_swap(self, s, lead):
        if s in self.through or lead in self.through:
            # a walk through s or lead changed: levels deeper than either's are wrong
            self.frm = min(self.frm, self.table_level(s, lead) + 1)

    def lookup(self, t, bits, i):
        """-> (leaf position, depth, root path bottom-up)"""
        if self.frm < 9:
            self.build(t)
        v = 0
        for k in range(8):
            v = (v << 1) | (bits[i + k] if i + k < len(bits) else 0)
        x, d = self.L[8][v]
        top = [self.L[j][v >> (8 - j)][0] for j in range(1, d + 1)]  # lane 64 - j in the kernel
        if t.body[x] & INNER:  # the code is longer than the tables reach
            self.cont += 1
            if d < 8:
                self.short += 1  # the tables stop short of depth 8 here: refresh them soon
                if self.short >= REFRESH:
                    self.frm = 0
            while t.body[x] & INNER:
                x = (t.body[x] & 255) * 2 + bits[i + d]
                d += 1
                top.append(x)
        return x, d, top[::-1]


def run(symbols):
    """Encode `symbols` with the path cache, then decode the bits with the prefix table and
    the path cache; assert every cached answer against the plain tree. Returns statistics."""
    t = Tree()
    pc = PathCache()
    bits = []
    for sym in symbols:
        fresh = t.where[sym] == 0
        if fresh:
            t.split(sym)
        x = t.where[sym]
        pv = pc.lookup(sym)
        true = t.path(x)
        if pv is None:
            probed = pc.probe(t, x)
            assert probed is None or probed == true, (sym, probed, true)
            pc.probes += probed is not None
            pv = true
            pc.insert(sym, pv)
        assert pv == true, (sym, pv, true)
        code = [p & 1 for p in reversed(pv)]
        bits += code[:-1] + [(sym >> k) & 1 for k in range(7, -1, -1)] if fresh else code
        t.update(x)
        for s, lead in t.swaps:
            pc.on_swap(s, lead)
    enc = dict(hits=pc.hits, misses=pc.misses, inval=pc.inval, probes=pc.probes)

    t = Tree()
    pt = LevelTables()
    i = 0
    out = []
    for _ in range(len(symbols)):
        x, d, pv = pt.lookup(t, bits, i)
        assert (x, d) == t.descend(bits, i) and pv == t.path(x)
        i += d
        if t.body[x] & NYT:
            sym = 0
            for k in range(8):
                sym = (sym << 1) | bits[i + k]
            i += 8
            t.split(sym)
            x = t.where[sym]
            pv = [x] + pv
        else:
            sym = t.body[x]
        assert pv == t.path(x)
        out.append(sym)
        t.update(x)
        for s, lead in t.swaps:
            pt.on_swap(s, lead)
    assert out == list(symbols) and i == len(bits)
    n = max(1, len(symbols))
    return dict(n=len(symbols), enc_hit=enc["hits"] / n, probe_hit=enc["probes"] / n, inval=enc["inval"] / n,
                rebuilds=pt.rebuilds / n, cont=pt.cont / n, bits=len(bits))


# ---- the kernels' update (hc_fgk.hip: update_fast / update_from / walk), on the same slot tree.
# The lane-parallel test works on the narrow weight words (weight << 10 | parent): a level is
# reported unless word(p + 1) >= word(p) + 1024, which never passes a non-leader and reports
# falsely only for the NYT's parent or a next position one heavier with a lower parent field.
# The walk does one exact level, then chases the climb back onto the known path (no leader
# test) and finishes the rest lane-parallel again.

def _word(t, p):
    return (t.w[p] << 10) | (t.up[p] if p < ROOT else 0) if p <= ROOT else (1 << 62)


def lanes_update(t, path, m=0):
    """update_from(path, m): path = positions of levels m.. (ROOT last); returns the first
    reported index or None (then every level incl. the root was incremented)"""
    k = None
    for j in range(m, len(path)):
        p = path[j]
        if p != ROOT and not _word(t, p + 1) >= _word(t, p) + 1024:
            k = j
            break
    for j in range(m, len(path) if k is None else k):
        t.w[path[j]] += 1
    return k


def kernel_walk(t, s, pv):
    """walk(s, pv): pv = the known root path, ROOT last"""
    while True:
        f = t.w[s]
        lead = s
        while t.w[lead + 1] == f:
            lead += 1
        if lead != s and lead != t.up[s]:
            a, c = t.body[s], t.body[lead]
            t.body[s], t.body[lead] = c, a
            t.relink(c, s)
            t.relink(a, lead)
            s = lead
        t.w[s] += 1
        c, td = t.up[s], []
        while c not in pv:
            td.append(c)
            c = t.up[c]
        path = td + pv[pv.index(c):]
        k = lanes_update(t, path)
        if k is None:
            return
        s, pv = path[k], path


def kernel_update(t, x, pv):
    """update_path: pv = t.path(x) + [ROOT]"""
    k = lanes_update(t, pv)
    if k is not None:
        kernel_walk(t, pv[k], pv)
