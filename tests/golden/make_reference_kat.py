"""Writes tests/golden/reference_kat.json: known-answer vectors transcribed from
the reference's own tests and hand-derived from its window code.

Every case cites the reference file:line it comes from. The reference's tests
drive a live server with SQL INSERTs; here each INSERT becomes one columnar
record: the GROUP BY column is dictionary-encoded to key_id, the event
timestamp (server publish time, Handler.hs:227-228) is any increasing value
inside one window/gap (the expected values do not depend on it), and the
aggregated / passthrough columns become value columns.
"""
import json
import os

COUNT_ALL, COUNT, SUM, MIN, MAX, AVG, LAST = range(7)
TUMBLING, HOPPING, SESSION, UNWINDOWED = range(4)
PER_RECORD, PER_BATCH, NONE = range(3)
I64, F64 = 0, 1

cases = []

# hstream/test/HStream/RegressionSpec.hs:42-56  (#394_SESSION)
# SELECT a, b, SUM(a) FROM s3 GROUP BY b, SESSION(INTERVAL 10 MINUTE) EMIT CHANGES;
# four INSERT (a, b) VALUES (1, 4)  ->  SUM(a) = 1, 2, 3, 4 ; a = 1 ; b = 4
cases.append({
    "name": "RegressionSpec#394_SESSION",
    "ref": "hstream/test/HStream/RegressionSpec.hs:42-56",
    "sql": "SELECT a, b, SUM(a) FROM s3 GROUP BY b, SESSION(INTERVAL 10 MINUTE) EMIT CHANGES;",
    "op": {"window_kind": SESSION, "emit_mode": PER_RECORD, "gap_ms": 600000,
           "col_types": [I64], "aggs": [[SUM, 0]]},
    "note": "passthrough a/b columns are constant here; session passthrough (HSG_LAST, merge keeps the existing session value) is covered by the seeded session parity tests",
    "batch": {"key_id": [0, 0, 0, 0], "ts": [1000, 1250, 1500, 1750], "cols": [[1, 1, 1, 1]]},
    "expect_changelog_aggs": [[1], [2], [3], [4]],
})

# hstream/test/HStream/RegressionSpec.hs:58-74  (#403_RAW)
# CREATE STREAM s5 AS SELECT SUM(a), a + 1, COUNT(*) AS result, b FROM s4 GROUP BY b EMIT CHANGES;
# four (1, 4) -> cnt 1..4, SUM(a) 1..4, a+1 = 2
cases.append({
    "name": "RegressionSpec#403_RAW",
    "ref": "hstream/test/HStream/RegressionSpec.hs:58-74",
    "sql": "SELECT SUM(a), a + 1, COUNT(*) AS result, b FROM s4 GROUP BY b EMIT CHANGES;",
    "op": {"window_kind": UNWINDOWED, "emit_mode": PER_RECORD,
           "col_types": [I64, I64], "aggs": [[SUM, 0], [LAST, 1], [COUNT_ALL, 0]]},
    "note": "column 1 carries the host-evaluated expression a + 1 (passthrough = LAST)",
    "batch": {"key_id": [0, 0, 0, 0], "ts": [1000, 1001, 1002, 1003], "cols": [[1, 1, 1, 1], [2, 2, 2, 2]]},
    "expect_changelog_aggs": [[1, 2, 1], [2, 2, 2], [3, 2, 3], [4, 2, 4]],
})

# hstream/test/HStream/RegressionSpec.hs:76-94  (HS352_INT, view)
# CREATE VIEW v6 as SELECT key1, key2, key3, SUM(key1) FROM s6 GROUP BY key1 EMIT CHANGES;
# rows key1 = 0,1,0,1,0 ; key2 = "hello_..0".."hello_..4" ; key3 = true,false,true,false,true
# SELECT * FROM v6 WHERE key1 = 1 -> SUM(key1) = 2, key2 = "hello_00000000000000000003", key3 = False
cases.append({
    "name": "RegressionSpec#HS352_INT",
    "ref": "hstream/test/HStream/RegressionSpec.hs:76-94",
    "sql": "CREATE VIEW v6 as SELECT key1, key2, key3, SUM(key1) FROM s6 GROUP BY key1 EMIT CHANGES;",
    "op": {"window_kind": UNWINDOWED, "emit_mode": NONE,
           "col_types": [I64, I64, I64], "aggs": [[LAST, 0], [LAST, 1], [LAST, 2], [SUM, 0]]},
    "note": "key2 strings dictionary-encoded to 0..4, key3 bools to 1/0; key_id 0 <-> key1 = 0, 1 <-> key1 = 1",
    "batch": {"key_id": [0, 1, 0, 1, 0], "ts": [1000, 1001, 1002, 1003, 1004],
              "cols": [[0, 1, 0, 1, 0], [0, 1, 2, 3, 4], [1, 0, 1, 0, 1]]},
    "expect_state": [[0, [0, 4, 1, 0]], [1, [1, 3, 0, 2]]],
})

# hstream/test/HStream/RunSQLSpec.hs:66-83  (GROUP BY without timewindow)
# SELECT SUM(a) AS result FROM s GROUP BY b EMIT CHANGES; (1,2),(2,2),(3,2),(4,3) -> 1, 3, 6, 4
cases.append({
    "name": "RunSQLSpec#GROUP_BY_without_timewindow",
    "ref": "hstream/test/HStream/RunSQLSpec.hs:66-83",
    "sql": "SELECT SUM(a) AS result FROM s GROUP BY b EMIT CHANGES;",
    "op": {"window_kind": UNWINDOWED, "emit_mode": PER_RECORD, "col_types": [I64], "aggs": [[SUM, 0]]},
    "batch": {"key_id": [0, 0, 0, 1], "ts": [1000, 1001, 1002, 1003], "cols": [[1, 2, 3, 4]]},
    "expect_changelog_aggs": [[1], [3], [6], [4]],
})

# hstream/test/HStream/RunSQLSpec.hs:140-157,178-189 (select from view)
# view: SELECT SUM(a) FROM (SELECT a, 1 AS b FROM source1) GROUP BY b
# insert a = 1, 2 -> SUM = 3 ; insert a = 3, 4 -> SUM = 10  (two polls = two batches)
cases.append({
    "name": "RunSQLSpec#select_from_view",
    "ref": "hstream/test/HStream/RunSQLSpec.hs:140-157,178-189",
    "sql": "CREATE VIEW v AS SELECT SUM(a) FROM source2 GROUP BY b EMIT CHANGES;",
    "op": {"window_kind": UNWINDOWED, "emit_mode": NONE, "col_types": [I64], "aggs": [[SUM, 0]]},
    "batches": [
        {"key_id": [0, 0], "ts": [1000, 1001], "cols": [[1, 2]], "expect_state": [[0, [3]]]},
        {"key_id": [0, 0], "ts": [5000, 5001], "cols": [[3, 4]], "expect_state": [[0, [10]]]},
    ],
})

# Hand-derived from windowsFor (hstream-processing/src/HStream/Processing/Stream/TimeWindowedStream.hs:105-117)
# and findSessions / aggregateProcessor (Store.hs:243-272, SessionWindowedStream.hs:84-118); SURVEY.md §8a.
windows = [
    {"ts": 100000, "size": 60000, "adv": 5000, "starts": list(range(45000, 100001, 5000))},
    {"ts": 3000, "size": 60000, "adv": 5000, "starts": [0]},
    {"ts": 59999, "size": 60000, "adv": 5000, "starts": list(range(0, 55001, 5000))},
    {"ts": -1, "size": 60000, "adv": 5000, "starts": []},
    {"ts": 10, "size": 7, "adv": 3, "starts": [6, 9]},
    {"ts": 13, "size": 7, "adv": 3, "starts": [9, 12]},
    {"ts": 12, "size": 7, "adv": 3, "starts": [6, 9, 12]},
    {"ts": 9999, "size": 10000, "adv": 10000, "starts": [0]},
    {"ts": 10000, "size": 10000, "adv": 10000, "starts": [10000]},
    {"ts": 0, "size": 10000, "adv": 10000, "starts": [0]},
]

cases.append({
    "name": "grace_24h_skips_expired_window",
    "ref": "TimeWindowedStream.hs:88-92, TimeWindows.hs:29-35",
    "op": {"window_kind": TUMBLING, "emit_mode": PER_RECORD, "size_ms": 10000,
           "col_types": [], "aggs": [[COUNT_ALL, 0]]},
    "note": "record 2 (ts 5000) arrives after stream time 200000000 >= 10000 + 86400000: window [0,10000) skipped",
    "batch": {"key_id": [0, 0, 0], "ts": [1000, 200000000, 5000], "cols": []},
    "expect_changelog": [[0, 0, 10000, [1]], [0, 200000000, 200010000, [1]]],
})

cases.append({
    "name": "session_gap10_merge",
    "ref": "SessionWindowedStream.hs:84-118, Store.hs:243-272",
    "op": {"window_kind": SESSION, "emit_mode": PER_RECORD, "gap_ms": 10, "col_types": [], "aggs": [[COUNT_ALL, 0]]},
    "batch": {"key_id": [0, 0, 0], "ts": [0, 20, 10], "cols": []},
    "expect_changelog": [[0, 0, 0, [1]], [0, 20, 20, [1]], [0, 0, 20, [3]]],
})
cases.append({
    "name": "session_gap10_split",
    "ref": "SessionWindowedStream.hs:84-118, Store.hs:243-272",
    "op": {"window_kind": SESSION, "emit_mode": PER_RECORD, "gap_ms": 10, "col_types": [], "aggs": [[COUNT_ALL, 0]]},
    "batch": {"key_id": [0, 0, 1, 1], "ts": [0, 11, 0, 10], "cols": []},
    "expect_changelog": [[0, 0, 0, [1]], [0, 11, 11, [1]], [1, 0, 0, [1]], [1, 0, 10, [2]]],
})

# hstream/test/HStream/RegressionSpec.hs:24-40  (#391_JOIN)
# SELECT s1.a, s2.a, s1.b, s2.b, SUM(s1.a), SUM(s2.a) FROM s1 INNER JOIN s2
#   WITHIN (INTERVAL 1 MINUTE) ON (s1.b = s2.b) GROUP BY s1.b EMIT CHANGES;
# INSERT INTO s1 (a, b) VALUES (1, 3); INSERT INTO s2 (a, b) VALUES (2, 3);
#   -> one row: SUM(s1.a) = 1, SUM(s2.a) = 2, s1.a = 1, s1.b = 3, s2.a = 2, s2.b = 3
# Codegen: s1 is the join's "this" stream (genStreamWithSourceStream,
# Codegen.hs:253-266), both windows 60000 ms (genJoinWindows :232-240), the
# join key is the ON field (genKeySelector :242-244), every source record's
# key is the dummy "{}" (HStore.hs:110-112: one record key, key_id 0), the
# joined value is genJoiner's union of prefixed fields (Internal/Codegen.hs:
# 62-67), then genGroupByNode's unwindowed aggregate over s1.b with the
# non-aggregate columns as passthrough (LAST, Codegen.hs:463-469).
joins = [{
    "name": "RegressionSpec#391_JOIN",
    "ref": "hstream/test/HStream/RegressionSpec.hs:24-40",
    "sql": "SELECT s1.a, s2.a, s1.b, s2.b, SUM(s1.a), SUM(s2.a) FROM s1 INNER JOIN s2 WITHIN (INTERVAL 1 MINUTE) "
           "ON (s1.b = s2.b) GROUP BY s1.b EMIT CHANGES;",
    "join": {"before_ms": 60000, "after_ms": 60000,
             "batches": [
                 {"side": [0], "key_id": [0], "join_key": [0], "ts": [1000], "handle": [0]},
                 {"side": [1], "key_id": [0], "join_key": [0], "ts": [1500], "handle": [1]}]},
    "note": "join_key 0 <-> b = 3; handle 0 = s1's record, 1 = s2's record",
    "values": {"0": {"a": 1, "b": 3}, "1": {"a": 2, "b": 3}},
    "expect_join_rows": [[0, 1, 0, 1500]],
    "group_by": ["this", "b"],
    "columns": [["this", "a"], ["other", "a"], ["this", "b"], ["other", "b"]],
    "op": {"window_kind": UNWINDOWED, "emit_mode": PER_RECORD, "col_types": [I64, I64, I64, I64],
           "aggs": [[LAST, 0], [LAST, 1], [LAST, 2], [LAST, 3], [SUM, 0], [SUM, 1]]},
    "expect_changelog_aggs": [[1, 2, 3, 3, 1, 2]],
}]

out = {
    "generator": "tests/golden/make_reference_kat.py",
    "reference": "Yu-zh/hstream @ 2025-01-17",
    "enums": {"agg": "COUNT_ALL=0 COUNT=1 SUM=2 MIN=3 MAX=4 AVG=5 LAST=6",
              "window": "TUMBLING=0 HOPPING=1 SESSION=2 UNWINDOWED=3",
              "emit": "PER_RECORD=0 PER_BATCH=1 NONE=2"},
    "windows_for": windows,
    "cases": cases,
    "joins": joins,
}
path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_kat.json")
with open(path, "w") as f:
    json.dump(out, f, indent=1)
print(path)
