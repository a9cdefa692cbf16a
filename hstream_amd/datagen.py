"""Synthetic columnar inputs for the BASELINE.json configs (C1–C5).

There is no dataset to download: every config is generated from a seed with
the shapes SURVEY.md §8d and BASELINE.md define:

  C1  tumbling 10 s COUNT(*), 1K keys, ts = 1.7e12 + i + U[0,500)
  C2  tumbling 60 s COUNT/SUM/AVG/MIN/MAX, 64K keys, ts = 1.7e12 + i*3.6e6/N + U[0,2000)
  C3  hopping 60 s / 5 s COUNT + SUM, 1M keys
  C4  session gap 30 s COUNT + SUM, 10M keys
  C5  tumbling 60 s SUM + MAX, Zipf(1.2) over a 1e8-key universe

``generate`` returns host numpy arrays (deterministic, used by the parity
tests and the CPU baseline); ``generate_torch`` draws the same distributions
directly into HBM with torch (used by bench.py so 100M-record inputs never
cross PCIe).
"""
from dataclasses import dataclass, field
from typing import List, Tuple

import numpy as np

from . import abi
from .columnar import OpSpec

TS0 = 1_700_000_000_000  # ms
HOUR = 3_600_000


@dataclass
class Config:
    name: str
    window_kind: int
    size_ms: int = 0
    advance_ms: int = 0
    gap_ms: int = 0
    keys: int = 1024
    n: int = 1_000_000
    col_type: int = abi.HSG_I64
    vrange: Tuple[float, float] = (-1e9, 1e9)
    aggs: List[Tuple[int, int]] = field(default_factory=list)
    ts_mode: str = "span"   # "span": near-sorted over one hour; "step": ts = TS0 + i + U[0,500)
    jitter: int = 2000
    zipf: float = 0.0       # > 0: Zipf(s) ranks over `keys` universe
    batch: int = 1 << 24
    seed: int = 0
    span_ms: int = HOUR     # "span" mode: event time covered by the config's `total` records

    def spec(self, emit_mode=abi.HSG_EMIT_PER_BATCH, state_capacity=0, out_capacity=0) -> OpSpec:
        ncols = 0 if all(k == abi.HSG_COUNT_ALL for k, _ in self.aggs) else 1
        return OpSpec(window_kind=self.window_kind, emit_mode=emit_mode, size_ms=self.size_ms,
                      advance_ms=self.advance_ms, gap_ms=self.gap_ms,
                      col_types=[self.col_type] * ncols, aggs=list(self.aggs),
                      state_capacity=state_capacity, out_capacity=out_capacity)


C_AGGS_FULL = [(abi.HSG_COUNT_ALL, 0), (abi.HSG_SUM, 0), (abi.HSG_AVG, 0), (abi.HSG_MIN, 0), (abi.HSG_MAX, 0)]

CONFIGS = {
    "C1": Config("C1", abi.HSG_TUMBLING, size_ms=10_000, keys=1000, n=1_000_000,
                 aggs=[(abi.HSG_COUNT_ALL, 0)], ts_mode="step", jitter=500, batch=1_000_000, seed=1),
    "C2": Config("C2", abi.HSG_TUMBLING, size_ms=60_000, keys=65_536, n=100_000_000,
                 aggs=C_AGGS_FULL, seed=2),
    "C2f": Config("C2f", abi.HSG_TUMBLING, size_ms=60_000, keys=65_536, n=100_000_000, col_type=abi.HSG_F64,
                  vrange=(0.0, 1e6), aggs=C_AGGS_FULL, seed=2),
    "C3": Config("C3", abi.HSG_HOPPING, size_ms=60_000, advance_ms=5_000, keys=1 << 20, n=1_000_000_000,
                 vrange=(-1e6, 1e6), aggs=[(abi.HSG_COUNT_ALL, 0), (abi.HSG_SUM, 0)], seed=3),
    "C4": Config("C4", abi.HSG_SESSION, gap_ms=30_000, keys=10_000_000, n=500_000_000,
                 aggs=[(abi.HSG_COUNT_ALL, 0), (abi.HSG_SUM, 0)], seed=4),
    "C5": Config("C5", abi.HSG_TUMBLING, size_ms=60_000, keys=100_000_000, n=100_000_000,
                 aggs=[(abi.HSG_SUM, 0), (abi.HSG_MAX, 0)], zipf=1.2, seed=5),
}


def _perm27(x):
    """Bijection on [0, 2^27): scatters Zipf ranks so hot keys land apart."""
    m = (1 << 27) - 1
    x = np.asarray(x, dtype=np.uint64) & np.uint64(m)
    for mul, add in ((0x9E3779B1, 0x7F4A7C15), (0x85EBCA77, 0x165667B1)):
        x = (x * np.uint64(mul | 1) + np.uint64(add)) & np.uint64(m)
        x ^= x >> np.uint64(13)
    return x


def zipf_ranks(rng, s, universe, n):
    out = np.empty(n, dtype=np.int64)
    filled = 0
    while filled < n:
        draw = rng.zipf(s, size=int((n - filled) * 1.1) + 16)
        draw = draw[draw <= universe]
        take = min(n - filled, draw.size)
        out[filled:filled + take] = draw[:take] - 1
        filled += take
    return out


def timestamps(cfg: Config, start: int, count: int, total: int, rng):
    i = np.arange(start, start + count, dtype=np.int64)
    if cfg.ts_mode == "step":
        base = TS0 + i
    else:
        base = TS0 + (i * cfg.span_ms) // max(1, total)
    return base + rng.integers(0, cfg.jitter, size=count, dtype=np.int64)


def generate(cfg: Config, n=None, start=0, total=None, seed=None):
    """Host arrays for records [start, start + n) of a config of `total` records."""
    n = cfg.n if n is None else n
    total = cfg.n if total is None else total
    rng = np.random.default_rng([cfg.seed if seed is None else seed, start])
    if cfg.zipf > 0:
        key = _perm27(zipf_ranks(rng, cfg.zipf, cfg.keys, n)).astype(np.uint32)
    else:
        key = rng.integers(0, cfg.keys, size=n, dtype=np.int64).astype(np.uint32)
    ts = timestamps(cfg, start, n, total, rng)
    lo, hi = cfg.vrange
    if cfg.col_type == abi.HSG_F64:
        v = np.round(rng.uniform(lo, hi, size=n), 3)
    else:
        v = rng.integers(int(lo), int(hi), size=n, endpoint=True, dtype=np.int64)
    return {"key_id": key, "ts": ts, "cols": [v]}


def generate_torch(cfg: Config, n, device="cuda", seed=None, start=0, total=None):
    """Same distributions drawn on the device (no PCIe). Zipf configs fall back
    to host generation + one copy (setup only, outside any timed region)."""
    import torch

    total = cfg.n if total is None else total
    if cfg.zipf > 0:
        h = generate(cfg, n=n, start=start, total=total, seed=seed)
        return {"key_id": torch.from_numpy(h["key_id"].view(np.int32)).to(device),
                "ts": torch.from_numpy(h["ts"]).to(device),
                "cols": [torch.from_numpy(h["cols"][0]).to(device)]}
    g = torch.Generator(device=device)
    g.manual_seed((cfg.seed if seed is None else seed) * 1_000_003 + start)
    key = torch.randint(0, cfg.keys, (n,), device=device, generator=g, dtype=torch.int64).to(torch.int32)
    i = torch.arange(start, start + n, device=device, dtype=torch.int64)
    if cfg.ts_mode == "step":
        base = TS0 + i
    else:
        base = TS0 + torch.div(i * cfg.span_ms, max(1, total), rounding_mode="floor")
    ts = base + torch.randint(0, cfg.jitter, (n,), device=device, generator=g, dtype=torch.int64)
    lo, hi = cfg.vrange
    if cfg.col_type == abi.HSG_F64:
        m = torch.round((torch.rand(n, device=device, generator=g, dtype=torch.float64) * (hi - lo) + lo) * 1000)
        # a tensor divisor: true division (a scalar one becomes a multiply by
        # its rounded reciprocal on the GPU), so every value is the double a
        # 3-decimal JSON literal parses to, as numpy's round(x, 3) gives
        v = m / torch.full_like(m, 1000.0)
    else:
        v = torch.randint(int(lo), int(hi) + 1, (n,), device=device, generator=g, dtype=torch.int64)
    return {"key_id": key, "ts": ts, "cols": [v]}
