"""Self-synchronisation of zstd sequence-bitstream decoding (measurement tool, not product).

Question: if a decoder starts the sequence section of a block at a wrong bit position and
with wrong FSE states, how many sequences does it take until its (bit position, LL, OF, ML
state) tuple meets the true trajectory?  If that is short against the block's sequence
count, the serial sequence chain of a block can be cut into segments decoded in parallel
from guessed entries (the decoder-side counterpart of K3's Jacobi segments).

Frames come from the oracle (byte-identical to the GPU encoder) on C3's mix chunks.
RFC 8878 §3.1.1.3.2 (sequences section), §4.1 (FSE tables).
"""
import os
import random
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import zh_testlib as T  # noqa: E402

LL_BITS = [0] * 16 + [1, 1, 1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16]
ML_BITS = [0] * 32 + [1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16]
LL_NORM = [4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1]
ML_NORM = [1, 4, 3, 2, 2, 2, 2, 2, 2] + [1] * 37 + [-1] * 7
OF_NORM = [1, 1, 1, 1, 1, 1, 2, 2, 2] + [1] * 15 + [-1] * 5


def build_dtable(norm, log):
    size = 1 << log
    high = size - 1
    sym = [0] * size
    nxt = {}
    for s, c in enumerate(norm):
        if c == -1:
            sym[high] = s
            high -= 1
            nxt[s] = 1
        elif c > 0:
            nxt[s] = c
    step = (size >> 1) + (size >> 3) + 3
    pos = 0
    for s, c in enumerate(norm):
        for _ in range(max(c, 0)):
            sym[pos] = s
            pos = (pos + step) & (size - 1)
            while pos > high:
                pos = (pos + step) & (size - 1)
    tab = []
    for u in range(size):
        s = sym[u]
        ns = nxt[s]
        nxt[s] += 1
        nb = log - (ns.bit_length() - 1)
        tab.append((s, nb, (ns << nb) - size))
    return tab


def read_ncount(buf, off, maxsv):
    bits = int.from_bytes(buf[off:off + 64], "little")
    bp = 0

    def get(k):
        return (bits >> bp) & ((1 << k) - 1)

    log = get(4) + 5
    bp = 4
    remaining = (1 << log) + 1
    thr = 1 << log
    nb = log + 1
    norm = []
    prev0 = False
    while remaining > 1 and len(norm) <= maxsv:
        if prev0:
            while True:
                r = get(2)
                bp += 2
                norm += [0] * r
                if r != 3:
                    break
        mx = (2 * thr - 1) - remaining
        v = get(nb)
        if (v & (thr - 1)) < mx:
            count = v & (thr - 1)
            bp += nb - 1
        else:
            count = v & (2 * thr - 1)
            if count >= thr:
                count -= mx
            bp += nb
        count -= 1
        remaining -= abs(count)
        norm.append(count)
        prev0 = count == 0
        while remaining < thr:
            nb -= 1
            thr >>= 1
    norm += [0] * (maxsv + 1 - len(norm))
    return norm, log, off + (bp + 7) // 8


def first_block_sequences(frame):
    """(stream bytes, nseq, (LL, OF, ML) tables and logs) of the frame's first compressed block."""
    p = 4
    fhd = frame[p]
    p += 1
    single = (fhd >> 5) & 1
    if not single:
        p += 1
    p += [0, 1, 2, 4][fhd & 3]
    p += [0 if not single else 1, 2, 4, 8][fhd >> 6]
    bh = int.from_bytes(frame[p:p + 3], "little")
    p += 3
    btype, bsize = (bh >> 1) & 3, bh >> 3
    if btype != 2:
        return None
    end = p + bsize
    b0 = frame[p]
    lt, sf = b0 & 3, (b0 >> 2) & 3
    if lt in (0, 1):
        if sf in (0, 2):
            hs, sz = 1, b0 >> 3
        elif sf == 1:
            hs, sz = 2, (b0 >> 4) + (frame[p + 1] << 4)
        else:
            hs, sz = 3, (b0 >> 4) + (frame[p + 1] << 4) + (frame[p + 2] << 12)
        p += hs + (sz if lt == 0 else 1)
    else:
        hs = [3, 3, 4, 5][sf]
        v = int.from_bytes(frame[p:p + hs], "little") >> 4
        bitsz = [10, 10, 14, 18][sf]
        csz = v >> bitsz
        p += hs + csz
    b0 = frame[p]
    if b0 < 128:
        nseq, p = b0, p + 1
    elif b0 < 255:
        nseq, p = ((b0 - 128) << 8) + frame[p + 1], p + 2
    else:
        nseq, p = frame[p + 1] + (frame[p + 2] << 8) + 0x7F00, p + 3
    modes = frame[p]
    p += 1
    tabs = []
    for (shift, dnorm, dlog, maxsv) in ((6, LL_NORM, 6, 35), (4, OF_NORM, 5, 31), (2, ML_NORM, 6, 52)):
        m = (modes >> shift) & 3
        if m == 0:
            tabs.append((build_dtable(dnorm, dlog), dlog))
        elif m == 1:
            tabs.append(([(frame[p], 0, 0)], 0))
            p += 1
        elif m == 2:
            norm, log, p = read_ncount(frame, p, maxsv)
            tabs.append((build_dtable(norm, log), log))
        else:
            return None
    return frame[p:end], nseq, tabs


class Stream:
    def __init__(self, s):
        self.v = int.from_bytes(s, "little")
        self.top = 8 * (len(s) - 1) + (s[-1].bit_length() - 1)

    def read(self, pos, k):
        """k bits below pos (zeros under bit 0)."""
        if k == 0:
            return 0
        lo = pos - k
        if lo >= 0:
            return (self.v >> lo) & ((1 << k) - 1)
        return (self.v << -lo) & ((1 << k) - 1)


def step(st, tabs, pos, s):
    (TL, _), (TO, _), (TM, _) = tabs
    eL, eO, eM = TL[s[0]], TO[s[1]], TM[s[2]]
    ofc, mb, lb = eO[0], ML_BITS[eM[0]], LL_BITS[eL[0]]
    pos -= ofc + mb + lb
    nL = eL[2] + st.read(pos, eL[1]); pos -= eL[1]
    nM = eM[2] + st.read(pos, eM[1]); pos -= eM[1]
    nO = eO[2] + st.read(pos, eO[1]); pos -= eO[1]
    return pos, (nL, nO, nM)


def trajectory(st, tabs, nseq):
    (_, kL), (_, kO), (_, kM) = tabs
    pos = st.top
    s = (st.read(pos, kL), st.read(pos - kL, kO), st.read(pos - kL - kO, kM))
    pos -= kL + kO + kM
    out = [(pos, s)]
    for _ in range(nseq - 1):
        pos, s = step(st, tabs, pos, s)
        out.append((pos, s))
    return out


def sync_distance(st, tabs, true_by_pos, p0, s0, limit):
    pos, s = p0, s0
    for n in range(limit):
        if true_by_pos.get(pos) == s:
            return n
        if pos < 0:
            return None
        pos, s = step(st, tabs, pos, s)
    return None


def main():
    nchunks = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    trials = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    data = T.gen(T.KINDS["mix"] if hasattr(T, "KINDS") else T.DG_MIX, nchunks, 0x5EED0003)
    rng = random.Random(1)
    res = []
    for c in range(nchunks):
        fr = T.oracle_frame(data[c * 65536:(c + 1) * 65536])
        fb = first_block_sequences(fr)
        if fb is None:
            continue
        sb, nseq, tabs = fb
        st = Stream(sb)
        tr = trajectory(st, tabs, nseq)
        (TL, _), (TO, _), (TM, _) = tabs
        ps, ss = tr[-1]
        end = ps - TO[ss[1]][0] - ML_BITS[TM[ss[2]][0]] - LL_BITS[TL[ss[0]][0]]
        assert end == 0, f"trajectory ends at bit {end}"
        by_pos = {p: s for p, s in tr}
        logs = tuple(t[1] for t in tabs)
        d_state, d_pos = [], []
        for _ in range(trials):
            # (a) the right bit position of a random sequence, wrong states
            i = rng.randrange(nseq // 4, nseq // 2)
            p = tr[i][0]
            s = tuple(rng.randrange(len(t[0])) for t in tabs)
            d_state.append(sync_distance(st, tabs, by_pos, p, s, nseq))
            # (b) a random bit position, states read from the bits there as if initial
            p = rng.randrange(st.top // 4, st.top // 2)
            s = (st.read(p, logs[0]), st.read(p - logs[0], logs[1]), st.read(p - logs[0] - logs[1], logs[2]))
            d_pos.append(sync_distance(st, tabs, by_pos, p - sum(logs), s, nseq))

        def summ(d):
            ok = sorted(x for x in d if x is not None)
            if not ok:
                return "never"
            return f"synced {len(ok)}/{len(d)} median {ok[len(ok) // 2]} p90 {ok[min(len(ok) - 1, int(0.9 * len(ok)))]} max {ok[-1]}"

        res.append((c, nseq, logs, summ(d_state), summ(d_pos)))
        print(f"chunk {c}: nseq {nseq} logs {logs} | right pos, wrong states: {summ(d_state)} | random pos: {summ(d_pos)}", flush=True)


if __name__ == "__main__":
    main()
