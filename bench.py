#!/usr/bin/env python3
"""Benchmark: windowed GROUP BY records/s on MI355X (BASELINE.json metric).

One step = one pass of the hot path over the configured workload: reset the
operator's HBM state, push every batch of the synthetic input through
libhstream_gpu and drain each batch's changelog into HBM. Default workload =
BASELINE config C2 (tumbling 60 s COUNT/SUM/AVG/MIN/MAX, 100M records, 64K
uniform keys, batches of 2^24), which fits one GPU.

`value` follows BASELINE.md's reporting formula ("records/s, end to end over
all batches, kernels plus H2D of the input"): the reference's operator is fed
host poll batches (Processor.hs:128-144), so every step hands its batches over
as pinned host buffers through hsg_push_batch_async; the library copies each
batch to HBM on the op's copy stream while the batch before it computes, so a
step costs max(PCIe, kernels). The batches use the ABI's narrow transport
(include/hstream_gpu.h hsg_enc: 16-bit key ids, ts as 16-bit offsets from
per-frame bases, the i64 value column as int32 -- C2's values are in
[-1e9, 1e9]; f64 columns of decimals as int32 mantissas), chosen per batch by
the product's hsg_batch_narrow, the pass the decoder (hsg_decode_json_batch)
runs on every batch it decodes; the library widens them on the device. The
narrowing runs before the timed region, as decoding does; its host rate is
reported (input_link.narrowed_by). The same JSON line also carries:
  hbm_resident  the same steps with the input already resident in HBM
                (hsg_push_batch on device columns): the kernels' own rate,
                with the batch pipeline's roofline;
  per_record    the EMIT CHANGES changelog the drop-in wires:
                one row per (record, window) in arrival order, HBM-resident
                input, its B_alg with the E*O changelog bytes.
`--input hbm` makes the HBM-resident run the headline (the kernels alone).

Multi-GPU: launched by torch.distributed.run, one process per GPU; every rank
ingests its own C2-sized slice from host memory (weak scaling) and the library
exchanges records by key hash over RCCL, so each GPU owns its key range's
state. Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
PCIE_PEAK_GBS = 63.0   # host link, PCIe Gen5 x16 (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--config", default="C2")
    p.add_argument("--records", type=int, default=0, help="records per rank per step (default: the config's N)")
    p.add_argument("--batch", type=int, default=0, help="records per push (default: the config's batch)")
    p.add_argument("--emit", default="per_batch", choices=["per_batch", "per_record", "none"])
    p.add_argument("--input", default="host", choices=["host", "hbm"],
                   help="headline input: pinned host batches, H2D timed (BASELINE.md), or HBM-resident")
    p.add_argument("--wide", action="store_true", help="host input at full width (no narrow transport)")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline time budget (0 = skip)")
    p.add_argument("--traffic-csv", default="", help="rocprofv3 --pmc counter CSV to fill roofline.traffic")
    p.add_argument("--force-exchange", action="store_true", help="N=1 through the RCCL exchange path")
    p.add_argument("--copy-drain", action="store_true", help="drain by copy instead of the registered changelog")
    p.add_argument("--no-hbm", action="store_true", help="skip the HBM-resident block (host headline only)")
    p.add_argument("--no-per-record", action="store_true", help="skip the per-record (EMIT CHANGES) block")
    p.add_argument("--state-capacity", type=int, default=0,
                   help="hsg_op_config state_capacity (default 0: the engine sizes the table itself)")
    p.add_argument("--extra-steps", type=int, default=3, help="timed steps of the hbm_resident / per_record blocks")
    p.add_argument("--no-sql-shape", action="store_true",
                   help="skip the sql_shape block (the SQL drop-in's op shape: literal forms + a passthrough)")
    p.add_argument("--sql-emit", default="both", choices=["both", "per_batch", "per_record"],
                   help="emit modes of the sql_shape block")
    p.add_argument("--only-sql", action="store_true",
                   help="profiling aid: only the sql_shape block (HBM-resident), no headline line")
    return p.parse_args()


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    from hstream_amd import abi, datagen
    from hstream_amd.engine import Engine, comm_unique_id

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    cfg = datagen.CONFIGS[args.config]
    n_rank = args.records or cfg.n
    batch = args.batch or min(cfg.batch, n_rank)
    emit = {"per_batch": abi.HSG_EMIT_PER_BATCH, "per_record": abi.HSG_EMIT_PER_RECORD,
            "none": abi.HSG_EMIT_NONE}[args.emit]

    comm_id = None
    if world > 1:
        idt = torch.zeros(abi.HSG_COMM_ID_BYTES, dtype=torch.uint8, device=dev)
        if rank == 0:
            idt.copy_(torch.frombuffer(bytearray(comm_unique_id()), dtype=torch.uint8))
        dist.broadcast(idt, 0)
        comm_id = bytes(idt.cpu().numpy().tobytes())
    elif args.force_exchange:
        comm_id = comm_unique_id()  # 1-rank communicator: the exchange path with itself
    eng = Engine(device=local, rank=rank, nranks=world, comm_id=comm_id, batch_capacity=batch)

    # time-window state: the engine sizes its HBM table itself (default, then
    # growth before any batch that could pass 3/4 load: hsg_op_config
    # state_capacity = 0), as a query with no cardinality hint; sessions: an
    # arena for at most one session per record
    groups = n_rank * world if cfg.window_kind == abi.HSG_SESSION else 0
    spec = cfg.spec(emit, state_capacity=args.state_capacity or groups)
    op = eng.op(spec)

    # synthetic input: this rank's slice of every step, drawn into HBM; every
    # global batch = world consecutive pieces of `batch` records, rank r
    # ingests piece r of each (the C3 layout: a contiguous 1/G of every batch)
    pieces = [(s, min(batch, n_rank - s)) for s in range(0, n_rank, batch)]
    parts = [datagen.generate_torch(cfg, m, device=dev, start=s * world + rank * m, total=cfg.n * world)
             for s, m in pieces]
    keys = torch.cat([p["key_id"] for p in parts])
    ts = torch.cat([p["ts"] for p in parts])
    cols = [torch.cat([p["cols"][0] for p in parts])] if spec.col_types else []
    del parts
    # the synthetic columns were produced on torch's stream, which the op's
    # stream is not ordered after (include/hstream_gpu.h, hsg_batch)
    torch.cuda.synchronize()

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    def timed(step, warmup, steps):
        for _ in range(warmup):
            step()
        barrier()
        st0 = op.stats()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        barrier()
        el = time.perf_counter() - t0
        st1 = op.stats()
        if world > 1:
            tt = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el = float(tt.item())
        return el, st0, st1

    if args.only_sql:
        # (profiling aid: the SQL op shape's kernels alone, e.g. for PMC traffic)
        op.close()
        sql = sql_shape_block(eng, cfg, keys, ts, cols, pieces, args)
        if rank == 0:
            print(json.dumps({"metric": "records/sec windowed GROUP BY (sql_shape only)", "value": None,
                              "config": {"workload": f"{cfg.name}: {workload_text(cfg)}"}, "sql_shape": sql}),
                  flush=True)
        eng.close()
        return
    dev_step = device_steps(op, keys, ts, cols, pieces, emit, args)
    hbm = None
    if args.input == "host":
        host_step, host_info = host_steps(op, keys, ts, cols, pieces, spec, emit, world, args)
        elapsed, st0, st1 = timed(host_step, args.warmup, args.steps)
        if not args.no_hbm:
            el_h, h0, h1 = timed(dev_step, 1, max(1, args.extra_steps))
            hbm = {"value": round(n_rank * world * max(1, args.extra_steps) / el_h, 1), "unit": "records/s",
                   "steps": max(1, args.extra_steps), "ms_per_step": round(el_h * 1e3 / max(1, args.extra_steps), 3),
                   "input": "HBM-resident device columns, one hsg_push_batch per batch",
                   "roofline": roofline(h0, h1, spec, emit)}
    else:
        host_info = None
        elapsed, st0, st1 = timed(dev_step, args.warmup, args.steps)

    total_records = n_rank * world * args.steps
    value = total_records / elapsed

    # roofline of the batch pipeline (HIP events on the op's stream; the same
    # kernels whichever way the input arrived)
    roof = roofline(st0, st1, spec, emit)
    traffic, tsrc = None, None
    if args.traffic_csv:
        traffic, tsrc = traffic_from_csv(args.traffic_csv, cfg, args.emit), args.traffic_csv
    else:
        traffic, tsrc = committed_traffic(args, world)
    roof["traffic"] = traffic
    roof["kernel"] = pipeline_name(cfg, args.emit)
    if tsrc:
        roof["traffic_source"] = tsrc
    agg_s = (st1["agg_kernel_ms"] - st0["agg_kernel_ms"]) / 1e3
    touched = st1["touched_total"] - st0["touched_total"]

    link = None
    if host_info is not None:
        h2d = host_info["bytes_per_step"] * args.steps
        xt = torch.tensor([float(h2d)], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(xt, op=dist.ReduceOp.SUM)
        gbs = float(xt[0]) / elapsed / 1e9
        link = {"bound": "pcie", "achieved": round(gbs, 3), "peak": PCIE_PEAK_GBS * world, "unit": "GB/s",
                "frac": round(gbs / (PCIE_PEAK_GBS * world), 4), "bytes_per_record": host_info["bytes_per_record"],
                "encoding": host_info["encoding"], "narrowed_by": host_info["narrowed_by"],
                "changelog_groups": host_info["groups"]}

    xchg = None
    if world > 1 or args.force_exchange:
        xb = st1["exchange_bytes"] - st0["exchange_bytes"]
        xs = (st1["exchange_ms"] - st0["exchange_ms"]) / 1e3
        xt = torch.tensor([float(xb), xs], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(xt, op=dist.ReduceOp.SUM)
        xb_all, xs_sum = float(xt[0]), float(xt[1])
        links = world * (world - 1) * 153e9  # xGMI: 7 links x ~153 GB/s per GPU, one per peer pair
        xchg = {"bytes_per_step": int(xb_all / args.steps), "device_ms_per_step_per_rank":
                round(xs_sum * 1e3 / args.steps / world, 3),
                "xgmi_frac": round(xb_all / elapsed / links, 6) if world > 1 else None}

    per_rec = None
    sql = None
    table_slots, grow_events = int(st1["table_slots"]), int(st1["grow_events"])
    if world == 1 and not args.force_exchange:
        del dev_step
        op.close()
        op = None
        if (not args.no_per_record and cfg.window_kind in (abi.HSG_TUMBLING, abi.HSG_UNWINDOWED)
                and emit != abi.HSG_EMIT_PER_RECORD):
            per_rec = per_record_block(eng, cfg, keys, ts, cols, pieces, args)
        if not args.no_sql_shape and cols and cfg.window_kind in (abi.HSG_TUMBLING, abi.HSG_UNWINDOWED):
            sql = sql_shape_block(eng, cfg, keys, ts, cols, pieces, args)

    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cpu = cpu_baseline(cfg, spec, args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": "records/sec windowed GROUP BY",
            "value": round(value, 1),
            "unit": "records/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64" if cfg.col_type == abi.HSG_F64 else "int64",
            "data": "synthetic",
            "config": {"workload": f"{cfg.name}: {workload_text(cfg)}", "records_per_gpu": n_rank,
                       "batch": batch, "keys": cfg.keys, "emit": args.emit,
                       "input": ("pinned host batches, H2D in the timed region (BASELINE.md reporting formula)"
                                 if args.input == "host" else "HBM-resident device columns"),
                       "parallelism": f"key-hash sharded x{world}" if world > 1 else "single GPU",
                       **({"state_capacity": args.state_capacity} if args.state_capacity else {})},
            "roofline": roof,
            "input_link": link,
            "cpu_baseline": cpu,
            "hbm_resident": hbm,
            "per_record": per_rec,
            "sql_shape": sql,
            "exchange": xchg,
            "agg_kernel_share": round(agg_s / elapsed, 4) if elapsed > 0 else None,
            "pairs_per_step": int((st1["pairs_total"] - st0["pairs_total"]) / max(1, args.steps)),
            "touched_per_step": int(touched / max(1, args.steps)),
            # HBM state table at the end of the run (slots of the time-window
            # table, or of the session key table) and its growth events
            "table_slots": table_slots,
            "table_grow_events": grow_events,
        }
        print(json.dumps(line), flush=True)
    if op is not None:
        op.close()
    eng.close()
    if world > 1:
        dist.destroy_process_group()


def device_steps(op, keys, ts, cols, pieces, emit, args):
    """One step over HBM-resident input: reset, then per batch one
    hsg_push_batch on device columns and one drain into HBM columns."""
    import ctypes as C
    import torch
    from hstream_amd import abi
    from hstream_amd.columnar import make_batch
    spec = op.spec
    out_cap = max(1, eng_out_capacity(op))
    dev = keys.device
    outs = {
        "key_id": torch.empty(out_cap, dtype=torch.int32, device=dev),
        "win_start": torch.empty(out_cap, dtype=torch.int64, device=dev),
        "win_end": torch.empty(out_cap, dtype=torch.int64, device=dev),
        "src_index": torch.empty(out_cap, dtype=torch.int64, device=dev),
        "aggs": [torch.empty(out_cap, dtype=torch.float64 if f else torch.int64, device=dev)
                 for f in spec.agg_is_f64()],
    }
    drain_dev = make_device_drain(op, outs, out_cap, zero_copy=not args.copy_drain)
    # batch descriptors over the HBM-resident slices, built once (the timed loop
    # is then one hsg_push_batch + one hsg_drain per batch)
    descs = [make_batch(keys[s:s + m], ts[s:s + m], [c[s:s + m] for c in cols], None, abi.HSG_MEM_DEVICE)
             for s, m in pieces]
    push_fn = op._lib.hsg_push_batch
    wm_c = C.c_int64(-1)

    def step():
        op.set_changelog(drain_dev.rows)  # (None with --copy-drain: the op's own buffer)
        op.reset()
        wm_c.value = -1
        for b, _keep in descs:
            rc = push_fn(op._h, C.byref(b), C.byref(wm_c))
            if rc != abi.HSG_OK:
                op._check(rc, "push_batch")
            if emit != abi.HSG_EMIT_NONE:
                drain_dev()
        return wm_c.value

    step.keep = (descs, outs, drain_dev)
    return step


def host_steps(op, keys, ts, cols, pieces, spec, emit, world, args):
    """BASELINE.md's reporting formula: each step hands every batch over as
    pinned host buffers (what a poll loop holds) through hsg_push_batch_async;
    the library queues each batch's H2D copies on the op's copy stream while
    the batch before it computes (op_prestage), so a step costs
    max(PCIe, kernels). Narrow transport unless --wide: the encoding is
    chosen here by hsg_batch_narrow (the decoder's pass), before any timing,
    as a decoder chooses it while decoding. The changelog goes into device columns
    registered for a group of batches and is drained after the group; a group
    is the whole step unless the step's worst-case rows exceed 96 GB of HBM
    (an asynchronous queue cannot be drained mid-way)."""
    import ctypes as C
    import numpy as np
    import torch
    from hstream_amd import abi
    from hstream_amd.columnar import make_batch
    from hstream_amd.ingest import _lib as ingest_lib
    L = ingest_lib()
    descs, host = [], []
    nbytes = 0
    encs = set()
    narrow_s = 0.0
    types = (C.c_int32 * max(1, len(spec.col_types)))(*spec.col_types)
    for s, m in pieces:
        # the batch as a decoder holds it (full width, pinned), then narrowed
        # in place by the product's hsg_batch_narrow -- the call
        # hsg_decode_json_batch makes on every batch it decodes
        pk = torch.empty(m, dtype=torch.int32).pin_memory()
        pt = torch.empty(m, dtype=torch.int64).pin_memory()
        pc = [torch.empty(m, dtype=c.dtype).pin_memory() for c in cols]
        pf = torch.empty(-(-m // abi.HSG_TS16_FRAME), dtype=torch.int64).pin_memory()
        pk.copy_(keys[s:s + m])
        pt.copy_(ts[s:s + m])
        for d, c in zip(pc, cols):
            d.copy_(c[s:s + m])
        b, keep = make_batch(pk.numpy().view(np.uint32), pt.numpy(), [c.numpy() for c in pc], None,
                             abi.HSG_MEM_HOST)
        if not args.wide:
            t0 = time.perf_counter()
            rc = L.hsg_batch_narrow(C.byref(b), C.cast(types, C.c_void_p), abi.HSG_NARROW_ALL, pf.data_ptr(), None,
                                    cpu_threads())
            narrow_s += time.perf_counter() - t0
            if rc != abi.HSG_OK:
                raise abi.HStreamGpuError(rc, "hsg_batch_narrow")
        descs.append(b)
        host.append((pk, pt, pc, pf, keep))
        kb = 2 if b.key_enc == abi.HSG_ENC_K16 else 4
        tb = {abi.HSG_ENC_TS16: 2, abi.HSG_ENC_TS32: 4}.get(b.ts_enc, 8)
        cb = [4 if b.col_enc[c] != abi.HSG_ENC_FULL else 8 for c in range(len(cols))]
        nbytes += (kb + tb + sum(cb)) * m + (pf.numel() * 8 if b.ts_enc == abi.HSG_ENC_TS16 else 0)
        tsn = {abi.HSG_ENC_TS16: "ts16", abi.HSG_ENC_TS32: "ts32"}.get(b.ts_enc, "ts64")
        encs.add(("k16" if kb == 2 else "k32") + "+" + tsn + "+" + ",".join(
            {abi.HSG_ENC_FULL: "full", abi.HSG_ENC_I32: "i32", abi.HSG_ENC_DEC32: "dec32"}[b.col_enc[c]]
            for c in range(len(cols))))
    n_rank = sum(m for _, m in pieces)
    wpr = -(-spec.size_ms // spec.advance_ms) if spec.window_kind == abi.HSG_HOPPING else 1
    row_bytes = 4 + 8 + 8 + 8 + 8 * len(spec.aggs)
    dev = keys.device
    state = {"cap": 0, "group": len(descs), "drain": None, "outs": None}

    def plan():
        # rows the library reserves per batch (op_push): n * ranks * wpr (per-batch
        # mode: capped by the table's capacity at the push, which the batches of
        # a step may grow, so the plan takes the uncapped worst case)
        per = [m * world * wpr for _, m in pieces]
        if emit == abi.HSG_EMIT_NONE:
            return 1, len(descs)
        budget = min(96 << 30, int(0.4 * torch.cuda.get_device_properties(dev).total_memory))
        g = len(descs)
        while g > 1 and max(per) * g * row_bytes > budget:
            g -= 1
        return max(per) * g, g

    def ensure(cap):
        if cap <= state["cap"]:
            return
        state["outs"] = None
        state["drain"] = None
        torch.cuda.empty_cache()
        outs = {"key_id": torch.empty(cap, dtype=torch.int32, device=dev),
                "win_start": torch.empty(cap, dtype=torch.int64, device=dev),
                "win_end": torch.empty(cap, dtype=torch.int64, device=dev),
                "src_index": torch.empty(cap, dtype=torch.int64, device=dev),
                "aggs": [torch.empty(cap, dtype=torch.float64 if f else torch.int64, device=dev)
                         for f in spec.agg_is_f64()]}
        state["outs"] = outs
        state["drain"] = make_device_drain(op, outs, cap, zero_copy=True, register=False)
        state["cap"] = cap

    lib = op._lib
    wm = C.c_int64(-1)
    no_cb = C.cast(None, abi.HSG_DONE_FN)  # no completion callback: hsg_op_wait below

    def step():
        cap, g = plan()
        ensure(cap)
        state["group"] = g
        if emit != abi.HSG_EMIT_NONE:
            op.set_changelog(state["drain"].rows)
        op.reset()
        wm.value = -1
        for i0 in range(0, len(descs), g):
            for b in descs[i0:i0 + g]:
                rc = lib.hsg_push_batch_async(op._h, C.byref(b), C.byref(wm), no_cb, None)
                if rc != abi.HSG_OK:
                    op._check(rc, "push_batch_async")
            rc = lib.hsg_op_wait(op._h)
            if rc != abi.HSG_OK:
                op._check(rc, "op_wait")
            if emit != abi.HSG_EMIT_NONE:
                state["drain"]()

    step.keep = (descs, host, state)
    info = {"bytes_per_step": nbytes, "bytes_per_record": round(nbytes / max(1, n_rank), 3),
            "encoding": sorted(encs), "groups": None,
            "narrowed_by": None if args.wide else
            f"hsg_batch_narrow (the decoder's own pass), {cpu_threads()} host threads: "
            f"{round(n_rank / max(narrow_s, 1e-9) / 1e6, 1)} M records/s"}

    class Info(dict):
        def __getitem__(self, k):
            if k == "groups":
                return -(-len(descs) // state["group"])
            return dict.__getitem__(self, k)
    return step, Info(info)


def roofline(st0, st1, spec, emit, valid_bytes=0, form_bytes=0):
    """Roofline of the batch pipeline: one "launch" = one batch through the
    partition + aggregation + changelog kernels, timed by HIP events on the
    op's stream (hsg_stats agg_kernel_ms). SURVEY.md 8(d) algorithmic bytes
      N*(4 + 8 + 8C) + 2*U*R + E*O
    N records, C value columns, U groups touched, R state row bytes (group key
    + slots, from the device's own slot program), E changelog rows, O row
    bytes (key 4, window 8 + 8, 8 per aggregate)."""
    from hstream_amd import abi
    launches = st1["agg_kernel_launches"] - st0["agg_kernel_launches"]
    agg_s = (st1["agg_kernel_ms"] - st0["agg_kernel_ms"]) / 1e3
    ncol = len(spec.col_types)
    rec_bytes = 4 + 8 + 8 * ncol + valid_bytes
    row_bytes = st1["state_row_bytes"]
    out_bytes = 4 + 8 + 8 + 8 * len(spec.aggs) + form_bytes if emit != abi.HSG_EMIT_NONE else 0
    touched = st1["touched_total"] - st0["touched_total"]
    pairs = st1["pairs_total"] - st0["pairs_total"]
    emitted = {abi.HSG_EMIT_PER_BATCH: touched, abi.HSG_EMIT_PER_RECORD: pairs}.get(emit, 0)
    owned = st1["records_owned"] - st0["records_owned"]
    alg_bytes = owned * rec_bytes + 2 * touched * row_bytes + emitted * out_bytes
    achieved = (alg_bytes / agg_s / 1e9) if agg_s > 0 else 0.0
    return {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": None,
            "state_row_bytes": row_bytes, "out_row_bytes": out_bytes,
            "alg_bytes_per_launch": int(alg_bytes / max(1, launches)),
            "rows_emitted_per_launch": int(emitted / max(1, launches)),
            "avg_launch_ms": round(agg_s * 1e3 / max(1, launches), 4)}


def per_record_block(eng, cfg, keys, ts, cols, pieces, args):
    """The EMIT CHANGES changelog (HSG_EMIT_PER_RECORD: one row per accepted
    (record, window) in arrival order, TimeWindowedStream.hs:89-103) over the
    same HBM-resident input; its B_alg counts the E*O changelog bytes."""
    import ctypes as C
    import torch
    from hstream_amd import abi
    from hstream_amd.columnar import make_batch
    emit = abi.HSG_EMIT_PER_RECORD
    spec = cfg.spec(emit)
    op = eng.op(spec)
    dev = keys.device
    cap = max(1, eng_out_capacity(op))
    outs = {"key_id": torch.empty(cap, dtype=torch.int32, device=dev),
            "win_start": torch.empty(cap, dtype=torch.int64, device=dev),
            "win_end": torch.empty(cap, dtype=torch.int64, device=dev),
            "src_index": torch.empty(cap, dtype=torch.int64, device=dev),
            "aggs": [torch.empty(cap, dtype=torch.float64 if f else torch.int64, device=dev) for f in spec.agg_is_f64()]}
    drain = make_device_drain(op, outs, cap, zero_copy=True)
    descs = [make_batch(keys[s:s + m], ts[s:s + m], [c[s:s + m] for c in cols], None, abi.HSG_MEM_DEVICE)
             for s, m in pieces]
    push_fn = op._lib.hsg_push_batch
    wm = C.c_int64(-1)

    def step():
        op.reset()
        wm.value = -1
        for b, _keep in descs:
            rc = push_fn(op._h, C.byref(b), C.byref(wm))
            if rc != abi.HSG_OK:
                op._check(rc, "push_batch")
            drain()

    torch.cuda.synchronize()
    step()
    torch.cuda.synchronize()
    k = max(1, args.extra_steps)
    st0 = op.stats()
    t0 = time.perf_counter()
    for _ in range(k):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    st1 = op.stats()
    n_rank = sum(m for _, m in pieces)
    roof = roofline(st0, st1, spec, emit)
    roof["kernel"] = pipeline_name(cfg, "per_record")
    host = None
    if args.input == "host":
        # the drop-in's mode with host input (BASELINE.md's formula): pinned
        # batches in the decoder's transport, H2D timed, rows into HBM
        del descs, outs, drain
        torch.cuda.empty_cache()
        hstep, hinfo = host_steps(op, keys, ts, cols, pieces, spec, emit, 1, args)
        hstep()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            hstep()
        torch.cuda.synchronize()
        elh = time.perf_counter() - t0
        gbs = hinfo["bytes_per_step"] * k / elh / 1e9
        host = {"value": round(n_rank * k / elh, 1), "unit": "records/s", "steps": k,
                "ms_per_step": round(elh * 1e3 / k, 3),
                "input": "pinned host batches, H2D in the timed region (BASELINE.md reporting formula)",
                "input_link": {"bound": "pcie", "achieved": round(gbs, 3), "peak": PCIE_PEAK_GBS, "unit": "GB/s",
                               "frac": round(gbs / PCIE_PEAK_GBS, 4),
                               "bytes_per_record": hinfo["bytes_per_record"], "encoding": hinfo["encoding"]}}
        del hstep
    if not (args.records or args.batch):
        # the committed PMC summary of this pipeline (tools/traffic.sh <cfg>_pr --emit per_record)
        import glob
        paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", f"traffic_{cfg.name.lower()}_pr.json")))
        if paths:
            with open(paths[-1]) as f:
                roof["traffic"] = int(json.load(f)["hbm_bytes_per_batch"])
            roof["traffic_source"] = os.path.relpath(paths[-1], ROOT)
    out = {"value": round(n_rank * k / el, 1), "unit": "records/s", "steps": k,
           "ms_per_step": round(el * 1e3 / k, 3), "emit": "per_record",
           "input": "HBM-resident device columns",
           "rows_per_step": int((st1["pairs_total"] - st0["pairs_total"]) / k), "roofline": roof,
           "host_input": host}
    op.close()
    torch.cuda.empty_cache()
    return out


def sql_shape_block(eng, cfg, keys, ts, cols, pieces, args):
    """The SQL drop-in's op shape on the same workload: the query hstream-sql's
    genGroupByNode dispatches for C2 -- `SELECT v, COUNT(*), SUM(v), AVG(v),
    MIN(v), MAX(v) FROM s GROUP BY key, TUMBLING (60 s)` -- whose objectSerde
    sink needs each value's Scientific literal form (HSG_OPF_LITERAL_FORMS:
    MIN / MAX tie words, the SUM's decimal count, Codegen.hs:436-461) and
    whose non-aggregate column `v` is a passthrough (HSG_LAST: the group's
    last record, Codegen.hs:463-469). The records carry validity bytes as a
    JSON decoder fills them (every field present; 1 in 16 literals decimal,
    e.g. `5.0`: bit 1). HBM-resident input, per batch and EMIT CHANGES, each
    with its roofline (B_alg adds the validity byte per record and the 4-byte
    form word per changelog row) and the path that ran (hsg_stats)."""
    import ctypes as C
    import torch
    from hstream_amd import abi
    from hstream_amd.columnar import OpSpec, make_batch
    dev = keys.device
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    valid = (1 + 2 * (torch.randint(0, 16, (keys.numel(),), device=dev, generator=g) == 0)).to(torch.uint8)
    aggs = [(abi.HSG_LAST, 0)] + list(cfg.aggs)
    modes = {"both": ("per_batch", "per_record")}.get(args.sql_emit, (args.sql_emit,))
    out = {"query": f"SELECT v, COUNT(*), SUM(v), AVG(v), MIN(v), MAX(v) GROUP BY key, {workload_text(cfg).split(' ')[0]}"
                    f" window (HSG_OPF_LITERAL_FORMS, v as HSG_LAST)",
           "valid": "every field present, 1 in 16 literals decimal (bit 1)", "input": "HBM-resident device columns"}
    k = max(1, args.extra_steps)
    n_rank = sum(m for _, m in pieces)
    torch.cuda.synchronize()
    for mode in modes:
        emit = abi.HSG_EMIT_PER_BATCH if mode == "per_batch" else abi.HSG_EMIT_PER_RECORD
        spec = OpSpec(window_kind=cfg.window_kind, emit_mode=emit, size_ms=cfg.size_ms, advance_ms=cfg.advance_ms,
                      col_types=[cfg.col_type], aggs=aggs, flags=abi.HSG_OPF_LITERAL_FORMS)
        op = eng.op(spec)
        cap = max(1, eng_out_capacity(op))
        outs = {"key_id": torch.empty(cap, dtype=torch.int32, device=dev),
                "win_start": torch.empty(cap, dtype=torch.int64, device=dev),
                "win_end": torch.empty(cap, dtype=torch.int64, device=dev),
                "src_index": torch.empty(cap, dtype=torch.int64, device=dev),
                "aggs": [torch.empty(cap, dtype=torch.float64 if f else torch.int64, device=dev)
                         for f in spec.agg_is_f64()],
                "form": torch.empty(cap, dtype=torch.int32, device=dev)}
        drain = make_device_drain(op, outs, cap, zero_copy=True)
        descs = [make_batch(keys[s:s + m], ts[s:s + m], [c[s:s + m] for c in cols], [valid[s:s + m]],
                            abi.HSG_MEM_DEVICE) for s, m in pieces]
        push_fn = op._lib.hsg_push_batch
        wm = C.c_int64(-1)

        def step():
            op.reset()
            wm.value = -1
            for b, _keep in descs:
                rc = push_fn(op._h, C.byref(b), C.byref(wm))
                if rc != abi.HSG_OK:
                    op._check(rc, "push_batch")
                drain()

        step()
        torch.cuda.synchronize()
        st0 = op.stats()
        t0 = time.perf_counter()
        for _ in range(k):
            step()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        st1 = op.stats()
        roof = roofline(st0, st1, spec, emit, valid_bytes=1, form_bytes=4)
        roof["kernel"] = ("SQL lean pipeline (k_part_hist_opt, offsets + decide, k_part_scatter_st with the "
                          "sequence word, k_agg_sql, k_sql_apply writing the changelog rows)" if mode == "per_batch"
                          else "per-record changelog (k_part_hist_opt, offsets + decide, stable k_part_scatter_st "
                               "with the sequence word, k_pr_bucket, k_pr_emit1)")
        tr = sql_traffic(cfg, mode)
        if tr:
            roof["traffic"], roof["traffic_source"] = tr
        batches = st1["batches"] - st0["batches"]
        out[mode] = {"value": round(n_rank * k / el, 1), "unit": "records/s", "steps": k,
                     "ms_per_step": round(el * 1e3 / k, 3), "roofline": roof,
                     "state_slots": int(st1["state_slots"]),
                     "lean_batches": int(st1["lean_batches"] - st0["lean_batches"]), "batches": int(batches),
                     "replays_onto_record_kernels": int(st1["replays"] - st0["replays"])}
        del descs, drain, outs
        op.close()
        torch.cuda.empty_cache()
    return out


def sql_traffic(cfg, mode):
    """Per-batch HBM bytes of the SQL op shape's pipeline on this config from
    the committed PMC summary (tools/gpu_r6_profile.sh ->
    profiles/<round>/traffic_<config>_sql[_pr].json), else None."""
    import glob
    name = f"traffic_{cfg.name.lower()}_sql{'_pr' if mode == 'per_record' else ''}.json"
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", name)))
    if not paths:
        return None
    with open(paths[-1]) as f:
        d = json.load(f)
    return int(d["hbm_bytes_per_batch"]), os.path.relpath(paths[-1], ROOT)


def workload_text(cfg):
    from hstream_amd import abi
    kind = {abi.HSG_TUMBLING: f"tumbling {cfg.size_ms // 1000}s", abi.HSG_HOPPING:
            f"hopping {cfg.size_ms // 1000}s/{cfg.advance_ms // 1000}s", abi.HSG_SESSION:
            f"session gap {cfg.gap_ms // 1000}s", abi.HSG_UNWINDOWED: "unwindowed"}[cfg.window_kind]
    names = {0: "COUNT(*)", 1: "COUNT", 2: "SUM", 3: "MIN", 4: "MAX", 5: "AVG", 6: "LAST"}
    aggs = "/".join(names[k] for k, _ in cfg.aggs)
    return f"{kind} {aggs}, {cfg.keys} keys{' zipf ' + str(cfg.zipf) if cfg.zipf else ' uniform'}"


def eng_out_capacity(op):
    # enough for the rows one batch can emit (per-batch: touched groups)
    from hstream_amd import abi
    spec = op.spec
    if spec.emit_mode == abi.HSG_EMIT_NONE:
        return 1
    return op.engine.batch_capacity * op.engine.nranks * (
        -(-spec.size_ms // spec.advance_ms) if spec.window_kind == abi.HSG_HOPPING else 1)


def make_device_drain(op, outs, cap, zero_copy=True, register=True):
    """Drain each batch's changelog into HBM-resident columns: registered with
    hsg_op_set_changelog (rows written in place, drain = count; register=False
    leaves the registration to the caller, through .rows) or, with
    --copy-drain, copied by hsg_drain from the op's own buffer."""
    import ctypes as C
    from hstream_amd import abi
    agg_ptrs = (C.c_void_p * max(1, len(outs["aggs"])))(*[t.data_ptr() for t in outs["aggs"]])
    rows = abi.hsg_rows(capacity=cap, mem=abi.HSG_MEM_DEVICE, n_aggs=len(outs["aggs"]),
                        key_id=outs["key_id"].data_ptr(), win_start=outs["win_start"].data_ptr(),
                        win_end=outs["win_end"].data_ptr(), src_index=outs["src_index"].data_ptr(),
                        aggs=C.cast(agg_ptrs, C.POINTER(C.c_void_p)),
                        form=outs["form"].data_ptr() if "form" in outs else None)
    got = C.c_uint64(0)
    if zero_copy:
        if register:
            op.set_changelog(rows)

        def drain_in_place():
            rc = op._lib.hsg_drain(op._h, None, C.byref(got))
            if rc != abi.HSG_OK:
                raise abi.HStreamGpuError(rc, "hsg_drain")
            return got.value

        drain_in_place.keep = (agg_ptrs, rows, outs)
        drain_in_place.rows = rows
        return drain_in_place

    def drain():
        rc = op._lib.hsg_drain(op._h, C.byref(rows), C.byref(got))
        if rc != abi.HSG_OK:
            raise abi.HStreamGpuError(rc, "hsg_drain")
        return got.value

    drain.keep = (agg_ptrs, rows, outs)
    drain.rows = None
    return drain


def pipeline_name(cfg, emit):
    """The kernels one bench "launch" (a batch, HIP events on the op's stream) covers."""
    from hstream_amd import abi
    if cfg.window_kind == abi.HSG_SESSION:
        if emit == "per_record":
            return ("session bucket replay (k_ss_phist, offsets, k_ss_pscatter, k_br_subhist, k_br_replay, "
                    "k_ss_reloc_copy, k_br_emit)")
        return "session merge (k_ss_phist, offsets, k_ss_pscatter, k_ss_sort, k_ss_apply)"
    if emit == "per_record":
        if cfg.window_kind in (abi.HSG_TUMBLING, abi.HSG_UNWINDOWED):
            return ("per-record changelog (k_part_hist_opt, offsets + decide, stable k_part_scatter_st, "
                    "k_pr_bucket, k_pr_emit1)")
        return ("per-record changelog (k_part_hist_opt, offsets + decide, stable k_part_scatter_st, "
                "k_pr_keysort, k_pr_offs, k_pr_keys)")
    if cfg.window_kind in (abi.HSG_TUMBLING, abi.HSG_UNWINDOWED):
        return ("batch pipeline (k_part_hist_opt, offsets + decide, k_part_scatter_st, k_agg_lean, "
                "k_pane_apply writing the changelog rows)")
    return "batch pipeline (k_part_hist_opt, offsets + decide, k_part_scatter_st, k_part_agg, k_touch_emit)"


def committed_traffic(args, world):
    """Per-batch HBM bytes of this configuration from the committed PMC summary
    (tools/traffic.sh -> profiles/<round>/traffic_<config>.json), when the run
    uses the configuration's default sizes; else None."""
    pr = args.emit == "per_record"  # the EMIT CHANGES lines: traffic_<config>_pr.json
    if world != 1 or args.batch or args.emit not in ("per_batch", "per_record") or args.force_exchange:
        return None, None
    if args.records and not pr:
        return None, None
    import glob
    suffix = "_pr" if pr else ""
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", f"traffic_{args.config.lower()}{suffix}.json")))
    if not paths:
        return None, None
    with open(paths[-1]) as f:
        d = json.load(f)
    # flags that only switch the extra blocks off measure the same pipeline
    extra = {"--no-host-input", "--no-per-record", "--no-hbm", "--no-sql-shape", "--input", "hbm"}
    words = [w for w in d.get("bench_args", "").split() if w not in extra]
    want = ["--config", args.config]
    if pr:
        want += ["--emit", "per_record"] + (["--records", str(args.records)] if args.records else [])
    if words not in (want, [] if not pr else None):
        return None, None
    return int(d["hbm_bytes_per_batch"]), os.path.relpath(paths[-1], ROOT)


def traffic_from_csv(path, cfg, emit):
    """HBM bytes per batch from a rocprofv3 --pmc counter_collection.csv that
    holds FETCH_SIZE and / or WRITE_SIZE rows: 2 x FETCH_SIZE (the gfx950
    correction for wide streaming reads, MI355X_MICROARCH.md) + WRITE_SIZE,
    over every hsg:: kernel, divided by the batches (dispatches of the
    pipeline's first kernel); KiB -> bytes."""
    import csv
    from hstream_amd import abi
    first = "k_ss_phist" if cfg.window_kind == abi.HSG_SESSION else (
        "k_pr_" if emit == "per_record" else "k_part_hist")
    fetch = write = 0.0
    batches = set()
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name", "")
            if "hsg::" not in name:
                continue
            if first in name:
                batches.add(r.get("Dispatch_Id"))
            cn, val = r.get("Counter_Name"), float(r.get("Counter_Value", 0))
            if cn == "FETCH_SIZE":
                fetch += val
            elif cn == "WRITE_SIZE":
                write += val
    if not batches:
        return None
    return int((2 * fetch + write) * 1024 / len(batches))


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_threads():
    """Host threads this process may use: its CPU affinity, at most 16 (the GPU
    box's CPU share per GPU; os.cpu_count() there reports the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def cpu_baseline(cfg, spec, seconds):
    """The oracle (sequential restatement of the reference path: ordered-map
    store) on a bounded sample of the same workload on this host:
    one thread, as the reference runs one query on one Haskell thread
    (Processor.hs:128-144), and key-partitioned over cpu_threads() threads
    (one oracle op per thread, records routed by key hash; each partition keeps
    its own stream time), the stronger CPU baseline SURVEY.md 8d asks for."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import pyoracle
    from concurrent.futures import ThreadPoolExecutor
    from hstream_amd import abi, datagen
    chunk = 1 << 18
    # sessions: the faithful store's findSessions scans every end time
    # (Store.hs:245-272, quadratic), so C4 is timed on its SURVEY.md 8d
    # sample, N = 5M / K = 100K (the same 50 records per key per hour)
    if cfg.window_kind == abi.HSG_SESSION and cfg.keys > 100_000:
        import dataclasses
        cfg = dataclasses.replace(cfg, keys=100_000, n=5_000_000)
        chunk = 1 << 14

    def run_single(budget):
        o = pyoracle.OracleOp(spec, faithful_sessions=True)
        done, wm, used = 0, -1, 0.0
        while used < budget and done < cfg.n:
            h = datagen.generate(cfg, n=chunk, start=done, total=cfg.n)
            t0 = time.perf_counter()
            wm = o.push(h["key_id"], h["ts"], h["cols"] if spec.col_types else [], None, watermark=wm)
            if spec.emit_mode != abi.HSG_EMIT_NONE:
                o.drain()
            used += time.perf_counter() - t0
            done += chunk
        o.close()
        return done, used

    def run_parallel(budget, T):
        ops = [pyoracle.OracleOp(spec, faithful_sessions=True) for _ in range(T)]
        wms = [-1] * T
        done, used = 0, 0.0

        def work(k, parts):
            key, ts, cols = parts[k]
            wms[k] = ops[k].push(key, ts, cols, None, watermark=wms[k])
            if spec.emit_mode != abi.HSG_EMIT_NONE:
                ops[k].drain()

        with ThreadPoolExecutor(T) as ex:
            while used < budget and done < cfg.n:
                h = datagen.generate(cfg, n=chunk * T, start=done, total=cfg.n)
                part = (h["key_id"].astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15) >> np.uint64(40)) % np.uint64(T)
                parts = []
                for k in range(T):
                    sel = part == k
                    parts.append((h["key_id"][sel], h["ts"][sel], [c[sel] for c in h["cols"]] if spec.col_types else []))
                t0 = time.perf_counter()
                list(ex.map(lambda k: work(k, parts), range(T)))
                used += time.perf_counter() - t0
                done += chunk * T
        for o in ops:
            o.close()
        return done, used

    n1, t1 = run_single(seconds)
    T = cpu_threads()
    nT, tT = run_parallel(seconds, T) if T > 1 else (n1, t1)
    return {"value": round(n1 / t1, 1), "unit": "records/s", "cores": 1, "kind": "port",
            "sample": f"first {n1} records of {cfg.name} (same generator, N={cfg.n}, K={cfg.keys}), "
                      f"oracle/hsoracle.cpp restatement ("
                      f"{'faithful end->key->start session store' if cfg.window_kind == abi.HSG_SESSION else 'ordered-map store'}"
                      f"), 1 thread",
            "cpu_model": cpu_model(), "host_cpus_visible": os.cpu_count(),
            "key_partitioned": {"value": round(nT / tT, 1), "unit": "records/s", "cores": T,
                                "sample": f"first {nT} records, {T} oracle ops, records routed by key hash"}}


if __name__ == "__main__":
    main()
