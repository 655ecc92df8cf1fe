"""Executable model of the adaptive decoder's parallel block-boundary pass (hc_adapt.hip
bounds_par_*), checked against the serial process in tests/test_adapt_model.py.

The reference finds block boundaries serially (revertAdaptRLE, transform.cpp:330-361): block k
is reverted by revertRLEBlock (transform.cpp:162-187) with a fresh MNP-5 machine until it has
produced exactly want_k bytes, and the next block starts at the following symbol. Errors: 13 a
count overshoots the block, 14 the symbols end inside a block, 15 symbols are left after the last.

The machine's state r (0..3: equal literals seen, 3 = the next symbol is a count) decides each
symbol's output length (count: the symbol, literal: 1). The parallel pass:

  1. no-reset trajectory: s0 = the machine's state run over the WHOLE stream without the block
     resets, len0 / O0 = its lengths and their exclusive prefix sums (a scan of 4-state
     transition functions and of lengths: parallel over chunks of symbols);
  2. Z: the positions p where a reset (state 0 at p) changes some symbol's LENGTH before the reset
     trajectory rejoins s0 (typically 1-2 symbols later). A block start outside Z changes no
     length: true output offsets there equal O0 + D, D the sum of the corrections so far;
  3. the scanner (one wave per stream) walks Z in order: z is a block start iff O0(z) + D is a
     block's first byte offset (a symbol of no-reset length 0 before z is in Z itself and is
     tested first, with the same offset); there the true
     machine is simulated from z until it rejoins s0, which gives the new D. Only these ~1-2 %
     of block starts form a serial chain;
  4. every chunk of symbols then runs the exact serial process from the entry the scanner
     predicts for it (state s0, output offset O0 + D; inside a simulated window: from the window's
     block start) and records its block starts, its first error and its exit (state, offset);
  5. verify: each chunk's entry must equal the previous chunk's exit (state and output offset:
     the whole state of the serial process); a chunk that does not is re-run from that exit,
     in order, until the entries agree. Chunk 0's entry is exact, so the result is exact by
     induction whatever the scanner predicted; the scanner only makes re-runs rare.
"""


def transition(s, x, xp):
    """transform.cpp:137-159 as a state machine (see hc_adapt.hip kFsmEq / kFsmNe)"""
    if s == 3:
        return 0
    return s + 1 if (s > 0 and x == xp) else 1


def length(s, x):
    return x if s == 3 else 1


def block_wants(W, H, B):
    per_row, nbr = -(-W // B), -(-H // B)
    return [min(B, W - bx * B) * min(B, H - by * B) for by in range(nbr) for bx in range(per_row)]


def serial(x, W, H, B):
    """the reference's serial process: (status, block starts)"""
    starts, pos, n = [], 0, len(x)
    for want in block_wants(W, H, B):
        starts.append(pos)
        got, s, prev = 0, 0, -1
        while got < want:
            if pos == n:
                return 14, starts
            c = x[pos]
            got += length(s, c)
            s = transition(s, c, prev)
            prev = c
            pos += 1
        if got != want:
            return 13, starts
    return (15 if pos != n else 0), starts


class Geometry:
    def __init__(self, W, H, B):
        self.W, self.H, self.B = W, H, B
        self.per_row, self.nbr = -(-W // B), -(-H // B)
        self.total = W * H

    def locate(self, o):
        """block k holding output offset o (k = nb at the end), its first offset E_k and want"""
        if o >= self.total:
            return self.per_row * self.nbr, self.total, 0
        rb = self.B * self.W
        by = min(o // rb, self.nbr - 1)
        sy = min(self.B, self.H - by * self.B)
        r = o - by * rb
        bx = min(r // (self.B * sy), self.per_row - 1)
        sx = min(self.B, self.W - bx * self.B)
        return by * self.per_row + bx, by * rb + bx * self.B * sy, sx * sy

    def is_start(self, o):
        k, e, _ = self.locate(o)
        return e == o


def walk(x, geo, q0, q1, s, o, record):
    """the exact serial process over symbols [q0, q1) entered in state s at output offset o:
    record(k, p) for every block k starting at p in range; returns (s, o, error, error_pos)"""
    n = len(x)
    k, e, want = geo.locate(o)
    got = o - e
    nb = geo.per_row * geo.nbr
    for p in range(q0, q1):
        if k >= nb:
            return s, o, 15, p
        if got == 0:
            record(k, p)
            s = 0
        c = x[p]
        ln = length(s, c)
        s = transition(s, c, x[p - 1] if p else -1)
        got += ln
        o += ln
        if got > want:
            return s, o, 13, p
        if got == want:
            k += 1
            got = 0
            want = geo.locate(o)[2] if k < nb else 0
    if q1 == n and k < nb:
        return s, o, 14, n
    return s, o, 0, q1


def parallel(x, W, H, B, chunk=64, win_cap=32):
    """the parallel pass: (status, block starts, stats)"""
    n = len(x)
    geo = Geometry(W, H, B)
    nb = geo.per_row * geo.nbr
    # 1. no-reset trajectory
    s0, len0, O0 = [0] * (n + 1), [0] * n, [0] * (n + 1)
    s = 0
    for i in range(n):
        s0[i] = s
        len0[i] = length(s, x[i])
        O0[i + 1] = O0[i] + len0[i]
        s = transition(s, x[i], x[i - 1] if i else -1)
    s0[n] = s
    # 2. Z: positions whose reset changes a length before rejoining s0
    Z = []
    for p in range(n):
        u, i, mism = 0, p, False
        while i < n and u != s0[i] and i - p < win_cap:
            if length(u, x[i]) != len0[i]:
                mism = True
            u = transition(u, x[i], x[i - 1] if i else -1)
            i += 1
        if mism or (i < n and u != s0[i]):  # unsynced within the cap: let the scanner simulate
            Z.append(p)
    # 3. scanner: D per chunk start, window overrides
    nch = -(-n // chunk) if n else 0
    D = 0
    entry = [None] * nch  # (q, s, o): chunk c starts its walk at symbol q in state s, offset o
    zi = 0
    c_next = 0
    hits = 0

    def close_chunks_until(pos):
        nonlocal c_next
        while c_next < nch and c_next * chunk <= pos:
            q = c_next * chunk
            entry[c_next] = (q, s0[q], O0[q] + D)
            c_next += 1

    while zi < len(Z):
        z = Z[zi]
        close_chunks_until(z)  # chunk starts up to z: outside every window, offset O0 + D
        o = O0[z] + D
        if o < geo.total and geo.is_start(o):
            hits += 1
            # simulate the true machine from z until it rejoins s0 (resets at block starts on
            # the way, overshoot / end: stop scanning, the chunk walks report it)
            k, e, want = geo.locate(o)
            got, u, i = 0, 0, z
            ok = True
            while True:
                if i > z and got == 0:
                    u = 0
                if i >= n or u == s0[i] and i > z:
                    break
                c = x[i]
                ln = length(u, c)
                u = transition(u, c, x[i - 1] if i else -1)
                got += ln
                o += ln
                if got > want:
                    ok = False
                    break
                if got == want:
                    k += 1
                    got = 0
                    want = geo.locate(o)[2] if k < nb else 0
                i += 1
                if c_next < nch and c_next * chunk == i and not (u == s0[i]):
                    # a chunk start inside the window: its walk runs in from the window's block
                    # start z (state 0, offset O0(z) + D)
                    entry[c_next] = ("from", z, O0[z] + D)
                    c_next += 1
            if not ok or i >= n:
                break
            D = o - O0[i]
            while zi < len(Z) and Z[zi] < i:
                zi += 1
            continue
        zi += 1
    close_chunks_until(n)
    while c_next < nch:
        q = c_next * chunk
        entry[c_next] = (q, s0[q], O0[q] + D)
        c_next += 1
    # 4. every chunk walks from its predicted entry (state, offset at its first symbol q; a
    # chunk starting inside a simulated window first runs in from the window's block start)
    starts = [None] * nb
    if nch == 0:
        return (0 if nb == 0 else 14), [], {"hits": 0, "reruns": 0, "Z": 0}
    res = []
    for c in range(nch):
        q = c * chunk
        if entry[c][0] == "from":
            s_q, o_q, _, _ = walk(x, geo, entry[c][1], q, 0, entry[c][2], lambda k, p: None)
        else:
            _, s_q, o_q = entry[c]
        rec = {}
        ex = walk(x, geo, q, min(n, (c + 1) * chunk), s_q, o_q, lambda k, p: rec.__setitem__(k, p))
        res.append(((s_q, o_q), ex, rec))
    # 5. verify in order: a chunk whose entry differs from the exact exit before it is re-run
    # from that exit (chunk 0's entry, state 0 at offset 0, is exact)
    reruns = 0
    status = 0
    exact = (0, 0)
    for c in range(nch):
        q = c * chunk
        ent, (s_out, o_out, err, ep), rec = res[c]
        if ent != exact:
            reruns += 1
            rec = {}
            s_out, o_out, err, ep = walk(x, geo, q, min(n, (c + 1) * chunk), exact[0], exact[1],
                                         lambda k, p: rec.__setitem__(k, p))
        for k, p in rec.items():
            starts[k] = p
        if err:
            status = err
            break
        exact = (s_out, o_out)
    got_starts = [p for p in starts if p is not None]
    return status, got_starts, {"hits": hits, "reruns": reruns, "Z": len(Z)}
