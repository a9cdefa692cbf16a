"""Mirror of hstream-sql's windowed GROUP BY dispatch (the codegen side only;
the BNFC parser/validator are out of scope).

  refine_interval    Interval refinement, hstream-sql/src/HStream/SQL/AST.hs:66-74
                     (DAY/WEEK/MONTH/YEAR multiply by 60*24, not 3600*24: kept)
  diff_time_to_ms    Internal/Codegen.hs:222-223
  gen_group_by_node  Codegen.hs:479-521 (+ genAggregateComponents :393-469,
                     genMaterialized :372-385): the window clause picks the
                     operator, the SELECT list the aggregate components.
                     HAVING is not applied to windowed GROUP BY (Codegen.hs:554-559)
                     and only one GROUP BY column exists (Validate.hs:556-562).
"""
from dataclasses import dataclass
from typing import List, Optional, Tuple, Union

from . import abi, processing as P

_UNIT_SECONDS = {
    "SECOND": 1,
    "MINUTE": 60,
    "DAY": 60 * 24,            # AST.hs:71 (sic)
    "WEEK": 60 * 24 * 7,       # AST.hs:72
    "MONTH": 60 * 24 * 30,     # AST.hs:73
    "YEAR": 60 * 24 * 365,     # AST.hs:74
}


def refine_interval(n: int, unit: str) -> int:
    """INTERVAL n UNIT -> seconds (DiffTime), as the reference refines it."""
    u = unit.upper().rstrip("S") if unit.upper() not in ("SECONDS",) else "SECOND"
    if u not in _UNIT_SECONDS:
        raise ValueError(f"unknown interval unit {unit}")
    if n <= 0:
        raise ValueError("Interval must be positive")  # Validate.hs:82-86
    return n * _UNIT_SECONDS[u]


def diff_time_to_ms(seconds: int) -> int:
    return int(seconds) * 1000  # picoseconds `div` 10^9


@dataclass(frozen=True)
class RTumblingWindow:
    seconds: int


@dataclass(frozen=True)
class RHoppingWindow:
    length: int
    hop: int


@dataclass(frozen=True)
class RSessionWindow:
    seconds: int


RWindow = Union[RTumblingWindow, RHoppingWindow, RSessionWindow]


@dataclass(frozen=True)
class RGroupBy:
    column: str
    window: Optional[RWindow] = None


# SELECT items: ("COUNT(*)",) / ("COUNT", col) / ("SUM", col) / ("MIN", col) /
# ("MAX", col) / ("AVG", col) / ("COL", col); optional alias as last element.
SelItem = Tuple


def gen_aggregate_components(sel: List[SelItem], float_fields=()) -> List[P.Agg]:
    out = []
    for item in sel:
        kind, *rest = item
        alias = None
        if kind == "COUNT(*)":
            if rest:
                alias = rest[0]
            out.append(P.COUNT_ALL(alias or "COUNT(*)"))
            continue
        col = rest[0]
        alias = rest[1] if len(rest) > 1 else None
        fl = col in float_fields
        if kind == "COUNT":
            out.append(P.COUNT(col, alias or f"COUNT({col})"))
        elif kind == "SUM":
            out.append(P.SUM(col, alias or f"SUM({col})", fl))
        elif kind == "MIN":
            out.append(P.MIN(col, alias or f"MIN({col})", fl))
        elif kind == "MAX":
            out.append(P.MAX(col, alias or f"MAX({col})", fl))
        elif kind == "AVG":
            # the reference throws "Unsupported aggregate function" (Codegen.hs:462);
            # this engine defines AVG = SUM(col) / COUNT(col)
            out.append(P.AVG(col, alias or f"AVG({col})", fl))
        elif kind == "COL":
            out.append(P.LAST(col, alias or col, fl))
        else:
            raise ValueError(f"Unsupported aggregate function: {kind}")
    return out


def gen_group_by_node(engine, sel: List[SelItem], group_by: RGroupBy, emit=abi.HSG_EMIT_PER_RECORD,
                      float_fields=(), state_capacity=0) -> P.Table:
    """genGroupByNode: groupBy -> (timeWindowedBy | sessionWindowedBy)? -> aggregate."""
    grouped = P.groupBy(engine, group_by.column)
    aggs = gen_aggregate_components(sel, float_fields)
    mat = P.Materialized(state_capacity=state_capacity)
    w = group_by.window
    if w is None:
        return grouped.aggregate(aggs, mat, emit)
    if isinstance(w, RTumblingWindow):
        return grouped.timeWindowedBy(P.mkTumblingWindow(diff_time_to_ms(w.seconds))).aggregate(aggs, mat, emit)
    if isinstance(w, RHoppingWindow):
        return grouped.timeWindowedBy(
            P.mkHoppingWindow(diff_time_to_ms(w.length), diff_time_to_ms(w.hop))).aggregate(aggs, mat, emit)
    if isinstance(w, RSessionWindow):
        return grouped.sessionWindowedBy(P.mkSessionWindows(diff_time_to_ms(w.seconds))).aggregate(aggs, mat, emit)
    raise ValueError("bad window")
