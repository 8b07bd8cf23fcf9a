"""bench.py — ringpop-node hot path on MI355X.

Workload (BASELINE.json configs[1], "C2"): a 10k-server HashRing (100 replica points, ~1M
tokens, built on the device) answering batched lookupN(key, 3) for 36-byte UUID-format keys.
One step = one device pass over one resident batch of 2^26 keys (default 15 steps ≈ 1.0B
lookups). Keys are synthetic (Philox UUID stream) and generated into HBM before
the timed region. With --gpus N every rank (one process per GPU) builds its own copy of the
ring and processes its own key stream: no data-path collective ("scaling": "weak").

Launch: `torchrun --nproc-per-node N bench.py --gpus N` (RANK / LOCAL_RANK / WORLD_SIZE from the
environment), or `python bench.py --gpus N`, which starts the N rank processes itself before
anything touches the GPU.

Printed (rank 0, one JSON line): value = lookupN(3)/s over all ranks, the dominant kernel's
roofline (48 algorithmic bytes per lookupN(3): 36 B key read + 12 B owner write),
the CPU oracle timed on this host as cpu_baseline, and the other configs' legs: C3 merge
(+ fold roofline, CPU baselines), C4 and C5 gossip simulations (+ traffic, per-round spread,
CPU baselines), the wire codec.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
BYTES_PER_LOOKUPN3 = 48  # 36 B key + 3 x 4 B owners
BYTES_PER_UPDATE = 49  # 16 B change + 16 B row read + 16 B row write + 1 B flag
METRIC = "ring lookups/s + member-updates merged/s; SWIM round time @100k members"


def load_pkg():
    import importlib.util
    spec = importlib.util.spec_from_file_location("ringpop_node_amd", os.path.join(REPO, "ringpop-node_amd", "__init__.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules["ringpop_node_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def _synth():
    import importlib.util
    spec = importlib.util.spec_from_file_location("rp_synth", os.path.join(REPO, "ringpop-node_amd", "synth.py"))
    S = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(S)
    return S


def _oracle():
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pyoracle
    return pyoracle


def c2_addr(i):
    return "10.%d.%d.%d:%d" % ((i >> 16) & 255, (i >> 8) & 255, i & 255, 20800 + i % 36)


def host_cores():
    """Host threads this job may use: the box's CPU share (OMP_NUM_THREADS, 16 per GPU on the
    pool) or the affinity mask."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(aff, int(omp))) if omp and omp.isdigit() else aff


def host_info():
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"cpu_model": model, "nproc": os.cpu_count(), "threads_used": host_cores()}


def pct(xs, q):
    return float(np.percentile(np.asarray(xs, dtype=np.float64), q)) if len(xs) else None


# ------------------------------------------------------------------ CPU baselines (oracle)

def cpu_baseline(servers, nkeys, threads, min_seconds=10.0):
    """The oracle (C restatement of lib/ring/index.js) on this host's cores: a bounded sample of
    the same workload (nkeys UUID keys, lookupN(key, 3)), repeated until >= min_seconds of wall;
    also one pass on one thread."""
    pyoracle = _oracle()
    ring = pyoracle.Ring(100)
    ring.add_remove(servers)
    keys = pyoracle.uuid_keys(42, 0, nkeys)
    n1 = max(1, nkeys // 16)
    t0 = time.perf_counter()
    ring.lookupn_keys(keys[:n1], 3, threads=1)
    one = n1 / (time.perf_counter() - t0)
    done, t0 = 0, time.perf_counter()
    while True:
        ring.lookupn_keys(keys, 3, threads=threads)
        done += nkeys
        dt = time.perf_counter() - t0
        if dt >= min_seconds:
            break
    return {"value": done / dt, "unit": "lookupN(3)/s", "cores": threads, "kind": "port",
            "value_1thread": one,
            "sample": "%d lookupN(key,3) (%d UUID keys x %d passes) on the same 10k-server ring, "
                      "oracle/orc_ring.c (farmhash32 + binary search + walk), %d pthreads, %.1f s; 1 thread: %d keys"
                      % (done, nkeys, done // nkeys, threads, dt, n1)}


def merge_cpu_baseline(n, k, threads):
    """C3 on the host: the oracle's Membership.update (oracle/orc_members.c: sequential fold +
    one checksum per batch, as lib/membership/index.js:249-324 runs) on one thread, and the fold
    sharded by id over `threads` threads with the checksum string formatted by all of them (the
    hash itself is one serial chain). `value` is the better of the two."""
    pyoracle = _oracle()
    S = _synth()
    names, st0, inc0 = S.c3_members(n)
    m = pyoracle.Members(names, local=names[0])
    m.set_ready(True)
    m.update_ids(np.arange(n, dtype=np.uint32), st0, inc0, now_ms=1)
    # every batch is fresh against the table (incarnations move forward 3 per batch), so every
    # batch applies most of its updates and pays the checksum, as the reference's benchmark does
    nb = 96
    batches = [S.c3_updates(n, k, seed=100 + b, base_inc=inc0 + 3 * b) for b in range(2 * nb)]
    L = pyoracle.lib()
    import ctypes
    L.orc_members_update_mt.restype = ctypes.c_uint32
    L.orc_members_update_mt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_uint32, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
    res = {}
    for label, T, b0 in (("1thread", 1, 0), ("all", threads, nb)):
        done, t0, b = 0, time.perf_counter(), b0
        while time.perf_counter() - t0 < 4.0 and b < b0 + nb:
            ids, us, ui = batches[b]
            if T == 1:
                m.update_ids(ids, us, ui, now_ms=1434500000000 + b)
            else:
                L.orc_members_update_mt(m.h, ids.ctypes.data, us.ctypes.data, ui.ctypes.data, k,
                                        1434500000000 + b, T, None)
            done += k
            b += 1
        dt = time.perf_counter() - t0
        res[label] = (done / dt, b - b0, dt)
    best = "all" if res["all"][0] >= res["1thread"][0] else "1thread"
    return {"value": res[best][0], "unit": "updates/s", "cores": threads if best == "all" else 1, "kind": "port",
            "value_1thread": res["1thread"][0], "value_all_threads": res["all"][0], "best_of": best,
            "sample": "C3 batches of %d updates over %d members incl. one checksum per batch: %d batches on 1 "
                      "thread (oracle/orc_members.c sequential fold) in %.1f s; %d batches with the fold sharded "
                      "by id over %d threads in %.1f s" % (k, n, res["1thread"][1], res["1thread"][2],
                                                            res["all"][1], threads, res["all"][2])}


def sim_cpu_baseline(n, kill_pct=1, seed=11, min_seconds=15.0, max_rounds=60, threads=1):
    """The simulator on this host: the oracle (oracle/orc_sim.c; the reference runs one view per
    process, this restatement runs every view) for as many rounds as fit in ~min_seconds."""
    pyoracle = _oracle()
    S = _synth()
    k = max(1, n * kill_pct // 100)
    names = [S.c2_addr(i) for i in range(n)]
    t0 = time.perf_counter()
    sim = pyoracle.Sim(names, S.c3_members(n)[2], S.kill_set(n, k, seed), seed=seed, susp_rounds=25,
                       now0=1434401518824 + 10 ** 9, threads=threads)
    create_s = time.perf_counter() - t0
    rounds, t0 = 0, time.perf_counter()
    while rounds < max_rounds:
        sim.step()
        rounds += 1
        if time.perf_counter() - t0 >= min_seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": dt * 1e3 / rounds, "unit": "ms/round", "cores": threads, "kind": "port",
            "create_s": create_s,
            "sample": "%d members, %d down: the first %d rounds of oracle/orc_sim.c on %d threads, %.1f s (+%.1f s "
                      "to create the views); early rounds are cheaper than the dissemination peak"
                      % (n, k, rounds, threads, dt, create_s)}


# ------------------------------------------------------------------ device legs

def merge_bench(rpa, torch, local, n=100_000, k=100_000, batches=512, warmup=3, world=1, dist=None,
                reduce_max=None, extras=True, part_log2=22):
    """C3 (BASELINE.json configs[2]): 100k-member table, a stream of batches of 100k updates (1%
    repeated addresses), Membership.update fold + one checksum per batch, inputs resident in HBM.
    Also: the fold alone (checksum deferred) against the HBM roofline at 49 B/update, the
    checksum chain alone, and the fold at a batch large enough not to be launch-bound.
    world > 1: every rank folds the whole stream on its own replica
    (DistMembership) and checksums the batches b % world == rank; the timed region is
    barrier-bracketed and the slowest rank's time is reported (strong scaling: the stream is
    fixed)."""
    S = _synth()
    names, st0, inc0 = S.c3_members(n)
    if world > 1:
        m = rpa.DistMembership(whoami=names[0], capacity=n, device=local, history_cap=batches + warmup + 64)
    else:
        m = rpa.Membership(whoami=names[0], capacity=n, device=local)
    ids0 = np.asarray(m.intern(names), dtype=np.uint32)
    m.update_ids(ids0, st0, inc0, now_ms=1)
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    # fresh batches (incarnations +3 per batch: most updates apply, every batch pays the
    # checksum), all resident in HBM before the timed region: 64 id/status sets, batch b takes
    # set b % 64 with its incarnations raised by 192 per lap (= inc0 + 3b + {-1, 0, +1}, as a
    # fresh c3_updates batch would have)
    nsets = 64
    sets = []
    for q in range(nsets):
        ids, us, ui = S.c3_updates(n, k, seed=100 + q, base_inc=inc0 + 3 * q)
        sets.append((torch.from_numpy(ids.view(np.int32)).cuda(), torch.from_numpy(us).cuda(),
                     torch.from_numpy(ui).cuda()))
    bufs = [(sets[b % nsets][0], sets[b % nsets][1], sets[b % nsets][2] + 3 * nsets * (b // nsets))
            for b in range(warmup + batches + 20)]
    app = torch.empty(k, dtype=torch.uint8, device="cuda")
    nst = torch.empty(k, dtype=torch.uint8, device="cuda")
    ninc = torch.empty(k, dtype=torch.int64, device="cuda")
    na = torch.zeros(1, dtype=torch.int32, device="cuda")

    def one(b, mm=m, bb=bufs, kk=k):
        d = bb[b % len(bb)]
        mm.update_dev(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), kk, 1434500000000 + b, app.data_ptr(),
                      nst.data_ptr(), ninc.data_ptr(), na.data_ptr(), sp)

    for b in range(warmup):
        one(b)
    m.local_checksum() if world > 1 else m.checksum
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(stream)
    for b in range(batches):
        one(warmup + b)
    # this replica's last checksum: every pending chain runs inside the timed region
    ck = m.local_checksum() if world > 1 else m.checksum
    e1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        dt = reduce_max([dt])[0]
        ck = m.latest_checksum()  # the last batch's checksum (gathered once, after the timed region)
    out = {"workload": "C3: %d-member table, %d updates/batch (1%% repeated addresses), fold + 1 checksum "
                       "per batch%s" % (n, k, ", %d replicas, batch-strided checksums" % world if world > 1 else ""),
           "n_gpus": world, "scaling": "strong", "batches": batches,
           "updates_per_s": k * batches / dt, "ms_per_batch": dt * 1e3 / batches,
           "gpu_ms_per_batch": e0.elapsed_time(e1) / batches, "checksum": ck,
           "note": "every batch applies most of its updates and its checksum string is built after it (written "
                   "by the blocks appended to the next batch's fold launch); the strings' serial farmhash chains "
                   "run in groups of 512 side by side (16 a workgroup) on a side stream, overlapping the next "
                   "batches' folds (2 groups of 512 slots within a 6 GiB pool, RP_MEMBERS_CK_BYTES); the last "
                   "batch's checksum is read inside the timed region, so "
                   "the final group's chains (one serial chain's latency, ~4.4 ms) are in the time: over "
                   "%d batches that drain adds ~%.1f us per batch" % (batches, 4400.0 / batches)}
    if world > 1 or not extras:  # the fold-only and large-batch legs are per-replica: rank 0's one-GPU run
        m.close()
        if world > 1 and extras:
            out["fold_large_partitioned"] = fold_large_part_bench(rpa, torch, S, local, world, dist, reduce_max,
                                                                  nb=1 << part_log2)
        return out
    # the fold alone (k_link + k_fold_fast + the gated sorted path), HIP events per batch on the
    # launch stream
    rpa.check(rpa.lib().rp_members_defer_checksum(m._h, 1))
    nf = 20
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(nf)]
    # a spin kernel ahead of the batches, so the host has enqueued them all before the GPU reaches
    # them: the events then time the device, not the host's launch rate (7 launches per batch take
    # the host longer than the GPU's 0.02 ms; without it the figure flips between 0.021 and 0.034)
    torch.cuda._sleep(4_000_000)
    for b in range(nf):
        evs[b][0].record(stream)
        one(warmup + batches + b)
        evs[b][1].record(stream)
    torch.cuda.synchronize()
    fold_ms = float(np.mean([a.elapsed_time(c) for a, c in evs]))
    rpa.check(rpa.lib().rp_members_defer_checksum(m._h, 0))
    # the checksum chain alone (string build + one farmhash over ~3.6 MB)
    t0 = time.perf_counter()
    for _ in range(5):
        m.compute_checksum()
    ck_ms = (time.perf_counter() - t0) * 1e3 / 5
    slen = len(m.generate_checksum_string())
    ach = BYTES_PER_UPDATE * k / (fold_ms * 1e-3) / 1e9
    out["fold"] = {"ms_per_batch": fold_ms, "bytes_per_update": BYTES_PER_UPDATE,
                   "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                "frac": ach / HBM_PEAK_GBS,
                                "note": "k_link + k_fold_fast + the gated sorted path (7 launches) per "
                                        "100k-update batch (HIP events); launch-bound at this batch size"}}
    out["checksum_chain"] = {"ms": ck_ms, "string_bytes": slen, "GBps": slen / (ck_ms * 1e-3) / 1e9,
                             "note": "one serial farmhash chain (not rooflined, SURVEY §8d)"}
    m.close()
    # a batch large enough that the fold is not launch-bound: 2^22 members, 2^22 updates
    nb = 1 << 22
    names_b = [c2_addr(i) for i in range(nb)]
    mb = rpa.Membership(whoami=names_b[0], capacity=nb, device=local)
    idb = np.asarray(mb.intern(names_b), dtype=np.uint32)
    incb = S.c3_members(nb)[2]
    mb.update_ids(idb, np.zeros(nb, np.uint8), incb, now_ms=1)
    rpa.check(rpa.lib().rp_members_defer_checksum(mb._h, 1))
    big = [tuple(torch.from_numpy(x).cuda() for x in (a.view(np.int32), s_, i_))
           for a, s_, i_ in [S.c3_updates(nb, nb, seed=300 + b, base_inc=incb + 3 * b) for b in range(7)]]
    app = torch.empty(nb, dtype=torch.uint8, device="cuda")
    nst = torch.empty(nb, dtype=torch.uint8, device="cuda")
    ninc = torch.empty(nb, dtype=torch.int64, device="cuda")
    one(0, mb, big, nb)
    torch.cuda.synchronize()
    def timed6(fn):
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(6)]
        torch.cuda._sleep(4_000_000)  # (as for the C3 fold above)
        for b in range(6):
            evs[b][0].record(stream)
            fn(b + 1)
            evs[b][1].record(stream)
        torch.cuda.synchronize()
        return float(np.mean([a.elapsed_time(c) for a, c in evs]))

    # separate status / incarnation output arrays (copies of the inputs, local overrides rewritten)
    copy_ms = timed6(lambda b: one(b, mb, big, nb))
    # the reference's own contract: evaluateUpdate rewrites the caller's update objects in place
    # (member.js), so the outputs are the input arrays (fresh incarnations +21: every batch
    # applies as the copy-out ones did)
    big2 = [(a, s_, i_ + 21) for a, s_, i_ in big]

    def inplace(b):
        d = big2[b % len(big2)]
        mb.update_dev(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), nb, 1434500000000 + 100 + b, app.data_ptr(),
                      d[1].data_ptr(), d[2].data_ptr(), na.data_ptr(), sp)

    big_ms = timed6(inplace)
    achb = BYTES_PER_UPDATE * nb / (big_ms * 1e-3) / 1e9
    out["fold_large"] = {"members": nb, "updates_per_batch": nb, "ms_per_batch": big_ms,
                         "updates_per_s": nb / (big_ms * 1e-3), "ms_per_batch_copy_out": copy_ms,
                         "outputs": "in place (the status / incarnation outputs are the input arrays, as the "
                                    "reference rewrites its update objects); ms_per_batch_copy_out: separate "
                                    "output arrays",
                         "roofline": {"bound": "hbm", "achieved": achb, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                      "frac": achb / HBM_PEAK_GBS}}
    mb.close()
    del big, big2, app, nst, ninc
    torch.cuda.empty_cache()
    return out


def fold_large_part_bench(rpa, torch, S, local, world, dist, reduce_max, nb=1 << 22):
    """The 2^22-update fold (fold_large) partitioned by member id over the ranks (PartMembership,
    SURVEY §8e's row partition): every rank holds the whole batch in HBM and folds the changes of
    its own 1/G of the ids (rp_members_update_range_dev: the scatter reads every change, writes
    and folds only its buckets'), in place, no checksum; HIP events per batch on each rank, the
    slowest rank's mean reported (strong scaling: the batch is fixed)."""
    names_b = [c2_addr(i) for i in range(nb)]
    mb = rpa.PartMembership(whoami=names_b[0], capacity=nb, device=local)
    idb = np.asarray(mb.intern(names_b), dtype=np.uint32)
    incb = S.c3_members(nb)[2]
    mb.update_ids(idb, np.zeros(nb, np.uint8), incb, now_ms=1)
    big = [tuple(torch.from_numpy(x).cuda() for x in (a.view(np.int32), s_, i_))
           for a, s_, i_ in [S.c3_updates(nb, nb, seed=300 + b, base_inc=incb + 3 * b) for b in range(7)]]
    app = torch.empty(nb, dtype=torch.uint8, device="cuda")
    na = torch.zeros(1, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream

    def one(b):
        d = big[b % len(big)]
        mb.update_dev(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), nb, 1434500000000 + b, app.data_ptr(),
                      d[1].data_ptr(), d[2].data_ptr(), na.data_ptr(), sp)

    one(0)
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(6)]
    dist.barrier()
    torch.cuda._sleep(4_000_000)  # (the host enqueues every batch before the GPU reaches them)
    for b in range(6):
        evs[b][0].record(stream)
        one(b + 1)
        evs[b][1].record(stream)
    torch.cuda.synchronize()
    ms = float(np.mean([a.elapsed_time(c) for a, c in evs]))
    ms = reduce_max([ms])[0]
    mb.close()
    del big, app
    torch.cuda.empty_cache()
    return {"members": nb, "updates_per_batch": nb, "n_gpus": world, "scaling": "strong", "ms_per_batch": ms,
            "updates_per_s": nb / (ms * 1e-3),
            "note": "each rank folds the changes of its own 1/%d of the member ids out of the whole batch "
                    "(outputs in place, no checksum); the slowest rank's mean over 6 batches" % world}


def sim_bench(rpa, torch, dist, local, n=10_000, kill_pct=1, seed=11, max_rounds=300, max_seconds=240.0, world=1,
              reduce_max=None):
    """C4 (BASELINE.json configs[3]) and C5 (configs[4]): n ringpop nodes with full views,
    kill_pct% down from the start, gossip rounds until convergence
    (scenario-runner.js:152-170 + every down member faulty everywhere). One GPU: one simulator
    handle. world > 1: the nodes are sharded by id range over the ranks and each round's four
    message exchanges are RCCL all-to-all-v (DistGossipSim); the timed region is bracketed by
    barriers and the max over ranks is reported. Reports rounds-to-convergence, wall time per
    round (mean, p50, p95, max and the worst round), exchange bytes and the traffic of §8d."""
    S = _synth()
    k = max(1, n * kill_pct // 100)
    names = [S.c2_addr(i) for i in range(n)]
    inc0 = S.c3_members(n)[2]
    dead = S.kill_set(n, k, seed)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if world > 1:
        sim = rpa.DistGossipSim(names, inc0, dead, seed=seed, suspicion_rounds=25, device=local)
    else:
        sim = rpa.GossipSim(names, inc0, dead, seed=seed, suspicion_rounds=25, device=local)
    torch.cuda.synchronize()
    create_s = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    rounds, conv, t0 = 0, False, time.perf_counter()
    per_round = []
    while rounds < max_rounds and time.perf_counter() - t0 < max_seconds:
        a = time.perf_counter()
        sim.step(1)
        c = sim.converged()  # syncs the round; collective when sharded (every rank leaves together)
        per_round.append(time.perf_counter() - a)
        rounds += 1
        if c:
            conv = True
            break
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    pr = np.asarray(per_round if per_round else [0.0])
    if world > 1:
        pr = np.asarray(reduce_max(list(pr)))  # round r's time = the slowest rank's
    dt, create_s = reduce_max([dt, create_s]) if world > 1 else (dt, create_s)
    ex_s, ex_dev = reduce_max([sim.exchange_s, sim.xchg.device_ms()]) if world > 1 else (0.0, 0.0)
    st = sim.stats()
    cnt = sim.counters()
    msg_bytes = 40 * cnt["messages"] + 24 * cnt["records"] + BYTES_PER_UPDATE * cnt["applied"]
    hashed = cnt["views_hashed"] * cnt["base_len"]
    out = {"workload": "%s: %d members, full views, %d down (%d%%), suspicion 25 rounds%s"
                       % ("C5" if n >= 100_000 else "C4", n, k, kill_pct,
                          ", nodes sharded over %d GPUs (RCCL all-to-all-v message exchange)" % world
                          if world > 1 else ", one GPU"),
           "n_gpus": world, "converged": conv, "rounds_to_convergence": rounds if conv else None,
           "rounds_run": rounds, "ms_per_round": dt * 1e3 / max(rounds, 1),
           "round_ms": {"p50": pct(pr * 1e3, 50), "p95": pct(pr * 1e3, 95), "max": float(pr.max() * 1e3),
                        "worst_round": int(pr.argmax())},
           "create_s": create_s, "stats": st,
           "traffic": {"messages": cnt["messages"], "records": cnt["records"], "applied": cnt["applied"],
                       "message_and_merge_bytes": msg_bytes,
                       "message_and_merge_GBps": msg_bytes / dt / 1e9,
                       "views_hashed": cnt["views_hashed"], "checksum_bytes_hashed": hashed,
                       "checksum_GBps": hashed / dt / 1e9,
                       "note": "bytes per SURVEY §8d: 40 B per message header + 24 B per change record sent + "
                               "49 B per applied update; checksum bytes = views re-hashed x the %d-byte "
                               "checksum string (serial chains: throughput, not a roofline)" % cnt["base_len"]}}
    if world > 1:
        out["exchange_bytes_per_round_rank0"] = sim.exchange_bytes / max(rounds, 1)
        # host time inside the message exchanges (counts all-to-all, inbox sizing, the byte
        # all-to-all-v queued on RCCL, join sums), the slowest rank's, per round
        out["exchange_ms_per_round"] = ex_s * 1e3 / max(rounds, 1)
        # the byte all-to-all-v kernels' own time on the device (RCCL; HIP events around each)
        out["exchange_device_ms_per_round"] = ex_dev / max(rounds, 1)
    sim.close()
    return out


def wire_bench(rpa, torch, dev, n_msgs=100_000, recs=32, reps=5):
    """Gossip wire bodies (rp_wire_*): n_msgs ping request bodies (ping-sender.js:71-76), each
    carrying `recs` issueAs change records (dissemination.js:163-170) over the C5 address set,
    encoded to JSON and decoded back on the device (records and the body headers a ping
    receiver reads: checksum, source, sourceIncarnationNumber). Reported as records/s and JSON GB/s (the
    bytes written by the encoder / read by the decoder; both are bounded by HBM)."""
    S = _synth()
    n = 100_000
    m = rpa.Membership(device=dev)
    m.intern([S.c2_addr(i) for i in range(n)])
    k = n_msgs * recs
    g = torch.Generator(device="cuda").manual_seed(5)
    ri = lambda hi, cnt, dt: torch.randint(0, hi, (cnt,), generator=g, device="cuda", dtype=dt)  # noqa: E731
    rec_off = torch.arange(0, k + 1, recs, device="cuda", dtype=torch.int32)
    addr, src = ri(n, k, torch.int32), ri(n, k, torch.int32)
    st = ri(4, k, torch.uint8)
    inc = ri(10 ** 7, k, torch.int64) + 1434401500000
    sinc = ri(10 ** 7, k, torch.int64) + 1434401500000
    ids = ri(16, k * 36, torch.uint8) + ord("a")
    ck, msrc = ri(2 ** 31, n_msgs, torch.int32), ri(n, n_msgs, torch.int32)
    msinc = ri(10 ** 7, n_msgs, torch.int64) + 1434401500000
    out_off = torch.empty(n_msgs + 1, dtype=torch.int64, device="cuda")
    L = rpa.lib()
    sp = torch.cuda.current_stream().cuda_stream
    args = [m._h, n_msgs, rec_off.data_ptr(), k, addr.data_ptr(), src.data_ptr(), st.data_ptr(), inc.data_ptr(),
            sinc.data_ptr(), ids.data_ptr(), 0, 1, ck.data_ptr(), msrc.data_ptr(), msinc.data_ptr()]
    rpa.check(L.rp_wire_encode_changes_dev(*args, None, out_off.data_ptr(), sp))
    total = int(out_off[-1].item())
    out = torch.empty(total, dtype=torch.uint8, device="cuda")
    rec_off2 = torch.empty(n_msgs + 1, dtype=torch.int32, device="cuda")
    e = lambda dt: torch.empty(k, dtype=dt, device="cuda")  # noqa: E731
    cols = [e(torch.int32), e(torch.int32), e(torch.uint8), e(torch.int64), e(torch.int64)]
    err = torch.empty(n_msgs, dtype=torch.int64, device="cuda")
    # the body headers a ping receiver reads (ping.js: checksum, source, sourceIncarnationNumber)
    h_ck, h_src = (torch.empty(n_msgs, dtype=torch.int32, device="cuda") for _ in range(2))
    h_sinc = torch.empty(n_msgs, dtype=torch.int64, device="cuda")

    def enc():
        rpa.check(L.rp_wire_encode_changes_dev(*args, out.data_ptr(), out_off.data_ptr(), sp))

    def dec():
        rpa.check(L.rp_wire_decode_changes_dev(m._h, out.data_ptr(), out_off.data_ptr(), n_msgs, rec_off2.data_ptr(),
                                               k, *[c.data_ptr() for c in cols], None, None, None, err.data_ptr(),
                                               h_ck.data_ptr(), h_src.data_ptr(), h_sinc.data_ptr(), sp))
        torch.cuda.synchronize()

    res = {}
    for name, fn in (("encode", enc), ("decode", dec)):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        res[name] = {"ms": dt * 1e3, "records_per_s": k / dt, "json_GBps": total / dt / 1e9}
    ok = bool((err == 0).all().item()) and bool(torch.equal(cols[0], addr)) and bool(torch.equal(cols[3], inc))
    ok = ok and bool(torch.equal(h_ck, ck)) and bool(torch.equal(h_src, msrc)) and bool(torch.equal(h_sinc, msinc))
    m.close()
    return {"workload": "%d ping request bodies x %d issueAs change records (C5 addresses), JSON encode + decode"
                        % (n_msgs, recs), "json_bytes": total, "round_trip_ok": ok, **res}


# The reference's own API per call on one core (tools/ref_node_bench.py): C2
# lookup 0.300 M/s, C2 lookupN(key, 3) 593 /s, C3 Membership.update of 100k + checksum 495 ms,
# computeChecksum alone at 100k members 200 ms.
REF_NODE = {"lookup_us": 1e6 / 0.300e6, "lookupN3_us": 1e6 / 593, "update_100k_batch_ms": 495.0,
            "computeChecksum_100k_ms": 200.0, "source": "BASELINE.md §3.1 (node v12, 1 core of the build container)"}


def api_latency_bench(timeout=300):
    """The drop-in JS API one call at a time, in node on this box (tools/api_latency.js):
    HashRing.lookup / lookupN (RingPop.lookup, index.js:434-471), lookupNBatch at 1 / 64 / 4096
    keys, and the drop-in Membership.update with 1 / 10 / 100 changes (the per-ping update,
    server/protocol/ping.js:44) at 100k / 10k / 1332 members, next to the reference's per-call
    times (REF_NODE)."""
    import shutil
    node = shutil.which("node")
    addon = os.path.join(REPO, "ringpop-node_amd", "js", "rpamd.node")
    if not node or not os.path.exists(addon):
        return {"skipped": "node or rpamd.node not available"}
    r = subprocess.run([node, os.path.join(REPO, "tools", "api_latency.js")], capture_output=True, text=True,
                       timeout=timeout)
    if r.returncode != 0:
        return {"error": r.stderr[-800:]}
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    out["reference_node_1core"] = REF_NODE
    b = out["lookupNBatch3"]
    # per-key device cost of a batched call against the reference's per-call lookupN(3)
    out["lookupN3_batch_where_device_wins"] = min((int(n) for n in b if b[n]["us_per_key"] < REF_NODE["lookupN3_us"]),
                                                  default=None)
    # the Node drop-in's default single call goes through the lookup service (serviceIdleMs 20)
    out["lookup_speedup_single_call"] = REF_NODE["lookup_us"] / out["lookup_service"]["median_us"]
    out["lookupN3_speedup_single_call"] = REF_NODE["lookupN3_us"] / out["lookupN3_service"]["median_us"]
    out["lookup_speedup_single_call_launch_per_call"] = REF_NODE["lookup_us"] / out["lookup"]["median_us"]
    return out


def pmc_traffic(keys, servers, nrep):
    """roofline.traffic for this line: the PMC-measured HBM bytes per key of the C2 lookupN(3)
    kernel (profiles/pmc_traffic.json, separate rocprofv3 --pmc passes) times this run's keys per
    step, labelled with the kernel and run they were measured on. None off the C2 shape (another
    server count or n), where no measurement exists."""
    p = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if not os.path.exists(p) or servers != 10000 or nrep != 3:
        return None, None
    with open(p) as f:
        d = json.load(f)
    per_key = d["lookupn_hbm_bytes_per_launch"] / d["keys_per_launch"]
    src = "%s; %.2f B/key measured over %d keys per launch (%s), scaled to %d keys" % (
        d.get("measured_on"), per_key, d["keys_per_launch"], d.get("kernel"), keys)
    return per_key * keys, src


# ------------------------------------------------------------------ launcher

def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(n):
    """`python bench.py --gpus N` without torchrun: start N fresh rank processes (one per GPU)
    before this process touches the GPU, wait, exit with the worst status."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    try:
        for p in procs:
            rc = max(rc, p.wait())
            if rc:
                break
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=15)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--ramp-ms", type=float, default=300.0,
                    help="after the W warmup steps, keep stepping (untimed) until this much warm-up time has "
                         "passed: the lookup kernel speeds up over its first ~15 launches (1.19 -> 0.90 ms) "
                         "while the device clocks ramp")
    ap.add_argument("--batch-log2", type=int, default=26)
    ap.add_argument("--servers", type=int, default=10000)
    ap.add_argument("--nrep", type=int, default=3)
    ap.add_argument("--cpu-keys", type=int, default=1 << 24)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-merge", action="store_true")
    ap.add_argument("--part-log2", type=int, default=22,
                    help="members and updates per batch (log2) of the partitioned fold leg at --gpus > 1")
    ap.add_argument("--merge-batches", type=int, default=2048,
                    help="C3 update batches in the timed stream (the final group's chains, one 4.4 ms chain latency, "
                         "are inside it: 2.1 us per batch at 2048, 8.6 at 512)")
    ap.add_argument("--no-wire", action="store_true")
    ap.add_argument("--no-api", action="store_true", help="skip the node per-call latency leg")
    ap.add_argument("--sim-n", type=int, default=10000, help="C4 members, one GPU (0: skip)")
    ap.add_argument("--sim5-n", type=int, default=100000, help="C5 members, sharded over all ranks (0: skip)")
    ap.add_argument("--sim5-cpu", type=int, default=1, help="time the C5 oracle sample (rank 0, N=1)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    assert world == args.gpus, "WORLD_SIZE=%d but --gpus %d" % (world, args.gpus)
    ndev = torch.cuda.device_count()
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, ndev)
    torch.cuda.set_device(local)
    backend = os.environ.get("RP_BENCH_BACKEND", "nccl")  # gloo: ranks sharing one GPU (tests)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    def reduce_max(vals):
        t = torch.tensor(vals, dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return [float(x) for x in t.cpu()]

    rpa = load_pkg()

    servers = [c2_addr(i) for i in range(args.servers)]
    t0 = time.perf_counter()
    ring = rpa.HashRing(device=local)
    ring.addRemoveServers(servers)
    build_ms = (time.perf_counter() - t0) * 1e3

    B = 1 << args.batch_log2
    nbuf = min(4, max(1, args.steps))
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    keys = [torch.empty(B * 36, dtype=torch.uint8, device="cuda") for _ in range(nbuf)]
    for j, kb in enumerate(keys):
        rpa.gen_uuid_keys_dev(42, (rank << 40) + j * B, B, kb.data_ptr(), sp)
    owners = torch.empty(B * args.nrep, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()

    def step(s):
        ring.lookupn_dev(keys[s % nbuf].data_ptr(), B, args.nrep, owners.data_ptr(), None, 36, None, sp)

    tw = time.perf_counter()
    for s in range(args.warmup):
        step(s)
    torch.cuda.synchronize()
    ramp = 0  # extra untimed steps until the clocks have ramped (--ramp-ms)
    while (time.perf_counter() - tw) * 1e3 < args.ramp_ms and ramp < 4096:
        for _ in range(4):
            step(args.warmup + ramp)
            ramp += 1
        torch.cuda.synchronize()
    if world > 1:
        ramp = int(reduce_max([ramp])[0])  # (ranks stop at their own time; report the largest)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.steps):
        ev[s][0].record(stream)
        step(s)
        ev[s][1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    elapsed, kern_ms = reduce_max([elapsed, kern_ms])

    total = B * args.steps * world
    del keys, owners
    torch.cuda.empty_cache()
    merge = None
    if not args.no_merge:
        merge = merge_bench(rpa, torch, local, batches=args.merge_batches, world=world, dist=dist,
                            reduce_max=reduce_max, part_log2=args.part_log2)
    sim5 = sim_bench(rpa, torch, dist, local, n=args.sim5_n, world=world, reduce_max=reduce_max) \
        if args.sim5_n else None
    if rank == 0:
        achieved = BYTES_PER_LOOKUPN3 * B / (kern_ms * 1e-3) / 1e9
        traffic, traffic_src = pmc_traffic(B, args.servers, args.nrep)
        out = {
            "metric": METRIC,
            "value": total / elapsed,
            "unit": "lookupN(3)/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "warmup_ramp_steps": ramp,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (Philox UUID-v4-format keys, C2 server addresses)",
            "config": {"workload": "C2: %d-server HashRing x 100 replica points, batched lookupN(n=%d) of "
                                   "36-byte keys, 2^%d keys per step" % (args.servers, args.nrep, args.batch_log2),
                       "servers": args.servers, "replica_points": 100, "tokens": ring.size,
                       "keys_per_step": B, "total_keys": total, "parallelism": "keys sharded, ring replicated"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_measured_on": traffic_src,
                         "kernel": "k_lookupn_lean<8,3,4> (+ k_lookupn_fix_tiles for deferred keys)",
                         "kernel_ms": kern_ms,
                         "bytes_per_unit": BYTES_PER_LOOKUPN3},
            "ring_build_ms": build_ms,
            "host": host_info(),
        }
        th = args.cpu_threads or host_cores()
        if merge is not None:
            out["merge"] = merge
            if not args.no_cpu and world == 1:
                out["merge"]["cpu_baseline"] = merge_cpu_baseline(100_000, 100_000, th)
        if args.sim_n and world == 1:
            out["sim"] = sim_bench(rpa, torch, dist, local, n=args.sim_n)
        if sim5:
            out["sim_c5"] = sim5
        if not args.no_wire:
            out["wire"] = wire_bench(rpa, torch, local)
        if not args.no_api and world == 1:
            out["api_latency"] = api_latency_bench()
        if not args.no_cpu and world == 1:
            out["cpu_baseline"] = cpu_baseline(servers, args.cpu_keys, th)
            if args.sim_n and "sim" in out:
                out["sim"]["cpu_baseline"] = sim_cpu_baseline(args.sim_n, threads=th)
            if sim5 and args.sim5_cpu:
                out["sim_c5"]["cpu_baseline"] = sim_cpu_baseline(args.sim5_n, threads=th, min_seconds=20.0)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
