"""Test oracle (CPU restatement) of the stream-stream join. Only tests/ may
import it.

Follows, record by record in arrival order over both streams:
  joinStreamProcessor   hstream-processing/src/HStream/Processing/Stream.hs:267-300
  joinStream            Stream.hs:222-250 (the other side swaps before/after,
                        and its joiner is flipped, so rows are always
                        (this value, other value))
  tksPut / tksRange     hstream-processing/src/HStream/Processing/Store.hs:334-385
                        (Map Int64 (Map k v): one entry per (ts, key), the last
                        put wins; the range includes its end points only when
                        the store holds some entry at both end timestamps)
  key selectors         hstream-sql/src/HStream/SQL/Codegen.hs:241-243 (a
                        missing join field throws at the first candidate,
                        which runTask catches: the record's scan ends there)
Pinned by the reference's one join vector, RegressionSpec.hs:24-40 (#391_JOIN,
tests/golden/reference_kat.json "joins", tests/test_join.py), and by
hand-derived vectors of its code (tests/test_join.py).
"""
import bisect

NONE = 0xFFFFFFFF


class JoinRef:
    def __init__(self, before_ms, after_ms):
        self.before, self.after = before_ms, after_ms
        self.stores = [dict(), dict()]   # side -> ts -> {key: (join key, handle)}
        self.ts_lists = [[], []]         # side -> sorted timestamps present

    def push_one(self, side, key, jkey, ts, handle):
        if key == NONE:
            return []
        st = self.stores[side]
        if ts not in st:
            st[ts] = {}
            bisect.insort(self.ts_lists[side], ts)
        st[ts][key] = (jkey, handle)
        other = 1 - side
        b, a = (self.before, self.after) if side == 0 else (self.after, self.before)
        lo, hi = ts - b, ts + a
        ost, tl = self.stores[other], self.ts_lists[other]
        inclusive = lo in ost and hi > lo and hi in ost
        if inclusive:
            i0, i1 = bisect.bisect_left(tl, lo), bisect.bisect_right(tl, hi)
        else:
            i0, i1 = bisect.bisect_right(tl, lo), bisect.bisect_left(tl, hi)
        out = []
        for t in tl[i0:i1]:
            c = ost[t].get(key)
            if c is None:
                continue
            cj, ch = c
            if jkey == NONE or cj == NONE:
                break
            if cj == jkey:
                out.append((handle, ch, jkey, max(ts, t)) if side == 0 else (ch, handle, jkey, max(ts, t)))
        return out

    def push(self, side, key, jkey, ts, handle):
        rows = []
        for i in range(len(side)):
            rows += self.push_one(int(side[i]), int(key[i]), int(jkey[i]), int(ts[i]), int(handle[i]))
        return rows

    def state_rows(self):
        return sum(len(m) for st in self.stores for m in st.values())
