"""Benchmark: batched CIF/CAF decode on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload cfg3|cfg4|cfg5|cfg2]
                    [--generator planted|uniform] [--mode eval|predict]

One step = one full decode (CifHr -> seeds -> CafScored -> seed loop / grow ->
force-complete -> NMS) of the rank's resident batch of synthetic fields, plus the packing
of its compact annotation records (pp_pack_compact) into pinned host memory (steps are
pipelined two deep: step k + 1 is enqueued before step k's records are waited for).  For
N > 1 each rank decodes its own batch (weak scaling, no data-path collective) and the
records of every rank are gathered to rank 0 over RCCL inside the step (the other ranks
pack into device memory and send from there).  Inputs are generated once and stay in HBM.

`--gpus N` without a torchrun environment starts the N rank processes itself (before any
GPU call in this process) and exits with their status.

Rank 0 prints ONE JSON line.  `roofline` is the CifHr accumulation of the metric: the
dense CifHr.accumulated map (pp_cifhr) of the same resident batch, timed with HIP events
on the launch stream; algorithmic bytes = 4*K*(5*H*W + H'*W') per image
over its launch time.  `roofline_decoder_cifhr` is the decoder's own block-sparse CifHr
stage inside `value` (its bytes: bench.cifhr_stage_bytes).
`cpu_baseline` is the oracle (oracle/pp_oracle.c, C restatement of the reference decoder)
on one host core, then on every CPU of the job's share, over bounded samples of the same
workload (planted, and a uniform leg); `cpu_baseline.twin` is the build's own C++ twin of the
decode (pp_decode_batch_cpu, csrc/decode_cpu.hip) on the same threads.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

WORKLOADS = {
    # BASELINE.json configs[2]: synthetic batch=256 at 80x80, full CifCaf, 1 GPU
    'cfg3': dict(h=80, w=80, batch=256, skeleton='coco', n_people=8),
    # configs[3]: batch 2048 at 80x80 over 8 GPUs = 256 per GPU, records gathered to rank 0
    'cfg4': dict(h=80, w=80, batch=256, skeleton='coco', n_people=8),
    # configs[1]: batch 1, CifHr + seeds only
    'cfg2': dict(h=80, w=80, batch=1, skeleton='coco', n_people=8, stages=3),
    # configs[4]: 160x160, dense 44-CAF skeleton, batch 512 over 8 GPUs = 64 per GPU
    'cfg5': dict(h=160, w=160, batch=64, skeleton='dense', n_people=16),
}
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=20)
    p.add_argument('--warmup', type=int, default=3)
    p.add_argument('--workload', default=None, choices=sorted(WORKLOADS),
                   help='default: cfg3 on one GPU, cfg4 on several')
    p.add_argument('--generator', default='planted', choices=('planted', 'uniform'))
    p.add_argument('--mode', default='eval', choices=('eval', 'predict'))
    p.add_argument('--batch', type=int, default=None, help='images per GPU (override)')
    p.add_argument('--cpu-seconds', type=float, default=18.0,
                   help='budget of the oracle CPU baseline sample (rank 0, N=1)')
    p.add_argument('--no-cpu-baseline', action='store_true')
    p.add_argument('--no-uniform', action='store_true',
                   help='skip the uniform-generator line added to the default run')
    p.add_argument('--no-predict', action='store_true',
                   help='skip the predict-defaults line added to the default run')
    p.add_argument('--no-multi', action='store_true',
                   help='skip the multi-scale (pp_decode_multi) lines added to the default run')
    p.add_argument('--backend', default='nccl', choices=('nccl', 'gloo'),
                   help='process group of N > 1 (gloo: rehearsal with several ranks on one '
                        'GPU, records staged through host memory)')
    p.add_argument('--no-configs', action='store_true',
                   help='skip the cfg2 / cfg5 lines added to the default run')
    p.add_argument('--stage-breakdown', action='store_true',
                   help='one library call per stage (per-stage times); implies --no-overlap')
    p.add_argument('--no-overlap', action='store_true',
                   help='run each step on one stream (no front / back half overlap of '
                        'consecutive steps, engine.DecodePipeline)')
    return p.parse_args()


def spawn_ranks(n):
    """Start bench.py once per GPU with the torchrun environment (RANK, LOCAL_RANK,
    WORLD_SIZE, MASTER_*) and wait for all of them; returns the worst exit status.  This
    process makes no GPU call (children are fresh processes, not re-execs)."""
    import signal
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    status = 0
    while procs:
        for p in list(procs):
            rc = p.poll()
            if rc is None:
                continue
            procs.remove(p)
            if rc != 0:
                status = status or rc
                for q in procs:  # one rank failed: the others would wait in a collective
                    q.send_signal(signal.SIGTERM)
        time.sleep(0.05)
    return status if status >= 0 else 128 - status


def log(msg):
    print('[bench {:.1f}s] {}'.format(time.perf_counter() - T_START, msg), file=sys.stderr,
          flush=True)


T_START = time.perf_counter()


def main():
    args = parse()
    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    import faulthandler
    faulthandler.enable()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    if world != args.gpus:
        raise SystemExit('--gpus {} but WORLD_SIZE {}'.format(args.gpus, world))
    # gloo rehearsal: ranks may share a GPU (nccl needs one GPU per rank)
    dev = torch.device('cuda', local_rank % max(1, torch.cuda.device_count())
                       if args.backend == 'gloo' else local_rank)
    torch.cuda.set_device(dev)
    comm_dev = dev if args.backend == 'nccl' else torch.device('cpu')
    if world > 1:
        if args.backend == 'nccl':
            dist.init_process_group('nccl', device_id=dev)
        else:
            dist.init_process_group('gloo')
        assert dist.get_world_size() == args.gpus
    if args.workload is None:
        args.workload = 'cfg3' if world == 1 else 'cfg4'

    from openpifpaf_amd import build as ppbuild
    # a no-op when the in-tree library is newer than its sources; otherwise only rank 0
    # builds, so ranks started together never link or load a half-written library
    if rank == 0:
        ppbuild.build(verbose=False)
    if world > 1:
        dist.barrier()
    from openpifpaf_amd import constants, synthetic
    from openpifpaf_amd.distributed import gather_packed
    from openpifpaf_amd._abi import (ANN_DTYPE, EVAL_CONFIG, PACK_ALL, PREDICT_CONFIG, make_config,
                                     packed_dtype)
    from openpifpaf_amd.engine import (STAGE_CAF, STAGE_CIFHR, STAGE_GROW, STAGE_SEEDS,
                                       DecodeEngine, DecodePipeline)

    wl = dict(WORKLOADS[args.workload])
    batch = args.batch or wl['batch']
    h, w = wl['h'], wl['w']
    skeleton = (constants.COCO_PERSON_SKELETON if wl['skeleton'] == 'coco'
                else constants.DENSE_DECODE_SKELETON)
    cfg = make_config(**(EVAL_CONFIG if args.mode == 'eval' else PREDICT_CONFIG))
    gen_kw = {'n_caf': len(skeleton)} if args.generator == 'uniform' else {
        'skeleton': skeleton, 'n_people': wl['n_people']}
    cif_h, caf_h = synthetic.batch(args.generator, batch, h, w, first_seed=rank * batch, **gen_kw)
    cif = torch.from_numpy(cif_h).to(dev)
    caf = torch.from_numpy(caf_h).to(dev)
    k = cif.shape[1]
    stages = wl.get('stages', 15)

    eng = DecodeEngine()
    stream = torch.cuda.current_stream()
    # default: consecutive steps overlap, the front half (CifHr, seeds, CafScored) of step
    # k + 1 beside the back half (seed loop, force-complete, NMS) of step k
    # (engine.DecodePipeline).  --no-overlap: CifHr alone, then the other stages in one
    # call; --stage-breakdown: one call per stage
    overlap = not (args.no_overlap or args.stage_breakdown) and stages == 15
    pipe = DecodePipeline(dev) if overlap else None
    # steps in flight on the host: one more than the pipeline's workspaces (3 with the
    # default two; a depth-3 pipeline needs 4, tools/pipe_gaps.py), 2 on one stream (two
    # output slots)
    depth = pipe.depth + 1 if overlap else 2
    groups = ((STAGE_CIFHR, STAGE_SEEDS, STAGE_CAF, STAGE_GROW) if args.stage_breakdown else
              (STAGE_CIFHR, STAGE_SEEDS | STAGE_CAF | STAGE_GROW))
    names = (('cifhr', 'seeds', 'caf_scored', 'grow_nms') if args.stage_breakdown else
             ('cifhr', 'seeds+caf', 'grow+nms') if overlap else ('cifhr', 'seeds+caf+grow+nms'))
    # event pairs per stage: the pipeline's five events (front stream: CifHr, the other
    # front stages; back stream: the back half), else one event between groups
    ev_pairs = ((0, 1), (1, 2), (3, 4)) if overlap else tuple(
        (i, i + 1) for i in range(len(groups)))
    # two event sets: with the two-deep pipeline, step k's events are read after step k + 1
    # has recorded its own
    ev_sets = [[torch.cuda.Event(enable_timing=True) for _ in range(max(5, len(groups) + 1))]
               for _ in range(depth)]

    comm = torch.cuda.Stream(device=dev) if world > 1 and args.backend == 'nccl' else None
    per_rank = []  # multi-rank: each rank's timings of the last timed_run (rank 0's view)
    counters = {'refetch_steps': 0, 'pack_bytes': 0}
    gather = {'steps': 0, 'verified_steps': 0, 'ranks_seen': world, 'full_record_steps': 0,
              'bytes': 0}

    def timed_run(cif, caf, steps, warmup, heads=None, skel=None, n_stages=None, run_cfg=None):
        """warmup + `steps` timed decode steps of one resident batch (cif / caf, or a
        multi-scale HeadSet) under `run_cfg` (default: the line's config): (elapsed s, max
        over ranks; per-group event ms per step; annotations decoded, on rank 0 those of all
        ranks)."""
        cfg_r = cfg if run_cfg is None else run_cfg
        skel = skeleton if skel is None else skel
        n_stages = stages if n_stages is None else n_stages
        k_img = heads.k if heads is not None else cif.shape[1]
        n_img = heads.n if heads is not None else cif.shape[0]
        compact = (k_img, len(skel), PACK_ALL)
        stage_ms = np.zeros(len(ev_pairs))
        # this rank's own view of the timed steps (the multi-rank line reports every rank's):
        # device ms from the step's first event to its last, host ms blocked on the records
        # (pack done), host ms inside the record gather
        rank_ms = {'decode': 0.0, 'records_wait': 0.0, 'gather': 0.0}

        def step(timed, k=0):
            """Enqueue one decode and its record fetch; returns (PendingRecords, events)."""
            ev = ev_sets[k % len(ev_sets)]
            if pipe is not None and n_stages == 15:
                b, pending = pipe.submit(cif, caf, skel, cfg_r, heads=heads, compact=compact,
                                         device_out=world > 1 and rank != 0,
                                         events=ev if timed else None)
                return b, (pending, ev)
            b = None
            for si, bits in enumerate(groups):
                if timed:
                    ev[si].record(stream)
                if n_stages & bits and heads is not None:
                    b = eng.launch_multi(heads, skel, cfg_r, stages=n_stages & bits)
                elif n_stages & bits:
                    b = eng.launch(cif, caf, skel, cfg_r, stages=n_stages & bits)
            if timed:
                ev[len(groups)].record(stream)
            # compact records -> pinned host memory (rank 0) or device memory (ranks that
            # send them to rank 0), enqueued behind the decode on a side stream
            pending = (eng.fetch_async(b, compact, device_out=world > 1 and rank != 0)
                       if n_stages & STAGE_GROW else None)
            return b, (pending, ev)

        def finish(step_out, timed, local=False):
            """Wait for one step's records (for N > 1: gathered to rank 0 over RCCL on the
            comm stream, which waits only for this step's pack)."""
            pending, ev = step_out
            n_recs = 0
            t_wait = time.perf_counter()
            if pending is None:
                torch.cuda.synchronize()
            elif world == 1 or local:
                recs, _ = pending.result()
                counters['refetch_steps'] += int(recs.dtype == ANN_DTYPE)
                counters['pack_bytes'] = len(recs) * recs.dtype.itemsize
                n_recs = len(recs)
            else:
                counts = pending.wait()
                t_gather = time.perf_counter()
                if timed:
                    rank_ms['records_wait'] += 1e3 * (t_gather - t_wait)
                if not pending.fits(int(counts.sum())):
                    raise SystemExit('record block too small after warmup')
                if comm is not None:
                    comm.wait_event(pending.done_event)
                # a pack that flagged PP_PACK_REFETCH sends the full records instead
                full = pending.refetch
                with torch.cuda.stream(comm) if comm is not None else torch.cuda.stream(None):
                    src = (pending.full_device_records() if full else
                           pending.device_records if rank != 0 else pending.host_records())
                width = (ANN_DTYPE if full else pending.dtype).itemsize
                if comm_dev.type == 'cpu':
                    src = src[:int(counts.sum()) * width].cpu()
                rep = {}
                recs, _ = gather_packed(src, counts, dist, n_max=n_img, dtype=pending.dtype,
                                        device=comm_dev, stream=comm, full=full, k=k_img,
                                        c=len(skel), report=rep)
                n_recs = len(recs) if recs is not None else 0
                if timed:
                    rank_ms['gather'] += 1e3 * (time.perf_counter() - t_gather)
                if rank == 0:
                    # every step's transfers are checked: each sender's digest of its record
                    # bytes against rank 0's digest of what arrived
                    gather['steps'] += 1
                    gather['verified_steps'] += int(rep['ranks_verified'] == world)
                    gather['ranks_seen'] = min(gather['ranks_seen'], rep['ranks_seen'])
                    gather['full_record_steps'] += int(rep['full_records'])
                    gather['bytes'] = rep['bytes']
            if timed:
                last = max(j for _, j in ev_pairs)
                ev[last].synchronize()
                for si, (i, j) in enumerate(ev_pairs):
                    stage_ms[si] += ev[i].elapsed_time(ev[j])
                rank_ms['decode'] += ev[0].elapsed_time(ev[last])
            return n_recs

        for _ in range(warmup):
            b, p = step(False)
            finish(p, False, local=True)  # sizes the record block (pack_cap)
        if warmup and depth > 1:
            # then `depth` + 1 steps in flight as the timed loop keeps them: the pinned record
            # blocks it needs at once are allocated here, not inside the clock (a 150 MB
            # pinned allocation of a uniform step blocks the host for up to 18 ms,
            # tools/host_pipe.py)
            pend = []
            for _ in range(depth + 1):
                b, p = step(False)
                pend.append(p)
                if len(pend) >= depth:
                    finish(pend.pop(0), False, local=True)
            while pend:
                finish(pend.pop(0), False, local=True)
        status = b.status.cpu().numpy()
        if status.any():
            raise SystemExit('decode status flags set: {}'.format(status[status != 0][:8]))
        if world > 1:
            b, p = step(False)
            finish(p, False)  # one gathered step before the clock (RCCL communicators)
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n_anns = 0
        # `depth` steps in flight: step k + depth - 1 is enqueued before step k's records are
        # waited for (decode outputs are double-buffered per workspace, engine.DecodeBuffers),
        # so the host's record handling and the next launches overlap the device work, and
        # with the overlapped pipeline the next front half is queued while the current back
        # half runs; every step's records are on rank 0's host before the clock stops
        inflight = []
        for k in range(steps):
            b, p = step(True, k)
            inflight.append(p)
            if len(inflight) >= depth:
                n_anns += finish(inflight.pop(0), True)
        while inflight:
            n_anns += finish(inflight.pop(0), True)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        if world > 1:
            # every rank's own numbers to rank 0 (for the line's per_rank list), then the
            # max over ranks of the wall clock
            mine = torch.tensor([elapsed, rank_ms['decode'] / steps,
                                 rank_ms['records_wait'] / steps, rank_ms['gather'] / steps],
                                dtype=torch.float64, device=comm_dev)
            every = torch.empty(world * 4, dtype=torch.float64, device=comm_dev)
            dist.all_gather_into_tensor(every, mine)
            per_rank[:] = [dict(zip(('elapsed_s', 'decode_ms_per_step',
                                     'records_wait_ms_per_step', 'gather_ms_per_step'),
                                    (round(float(v), 4) for v in row)), rank=r)
                           for r, row in enumerate(every.cpu().numpy().reshape(world, 4))]
            elapsed = max(p['elapsed_s'] for p in per_rank)
        return elapsed, stage_ms / steps, n_anns

    log('rank {}/{}: {} on {}'.format(rank, world, args.workload, dev))
    elapsed, stage_avg, n_anns = timed_run(cif, caf, args.steps, args.warmup)
    log('main workload done')

    images = batch * world * args.steps
    value = images / elapsed
    ms_step = 1e3 * elapsed / args.steps
    hh, ww = (h - 1) * 8 + 1, (w - 1) * 8 + 1
    cifhr_bytes, hr_tiles, sector_bytes = cifhr_stage_bytes(cif_h, 8, cfg.cif_threshold,
                                                            cfg.seed_threshold)
    achieved = cifhr_bytes / (stage_avg[0] * 1e-3) / 1e9
    if world > 1 and args.backend == 'gloo':
        # the rehearsal's ranks share one GPU: 8 ranks x two 14.3 GB workspaces fill most of
        # its 288 GB, so the decode workspaces go before the dense map's 9.6 GB per rank
        # (memory budget)
        import gc
        pipe, eng = None, None
        gc.collect()
        torch.cuda.empty_cache()
        dist.barrier()
    dense_ms = dense_cifhr_ms(cif, cfg, stream, args.steps, args.warmup)
    dense_bytes = 4 * k * (5 * h * w + hh * ww) * batch  # SURVEY.md §8d, per launch
    dense_gbs = dense_bytes / (dense_ms * 1e-3) / 1e9
    line = {
        'metric': 'decoder images/sec + ms/image, 17-CIF/19-CAF @80x80; CifHr HBM GB/s vs '
                  'roofline',
        'value': round(value, 1),
        'unit': 'images/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': round(ms_step, 4),
        'ms_per_image': round(ms_step / (batch * world), 6),
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'f32',
        'data': 'synthetic ({} generator, fields resident in HBM)'.format(args.generator),
        'config': {
            'workload': '{}: {} images/GPU at {}x{}, 17 CIF / {} CAF, full CifCaf decode, {} '
                        'defaults'.format(args.workload, batch, h, w, len(skeleton), args.mode),
            'global_batch': batch * world,
            'parallelism': 'image-sharded dp{} (compact records gathered to rank 0, {} '
                           'send/recv)'.format(world, 'RCCL' if args.backend == 'nccl' else
                                               'gloo rehearsal, ranks sharing GPUs')
                           if world > 1 else 'single GPU',
        },
        # the hand-over format: compact records (pp_pack_compact) instead of 1544-byte pp_ann
        'records': {
            'record_bytes': packed_dtype(k, len(skeleton), PACK_ALL).itemsize,
            'full_record_bytes': ANN_DTYPE.itemsize,
            'bytes_per_step_rank0': counters['pack_bytes'],
            'refetch_steps': counters['refetch_steps'],
        },
        'stage_ms': {n: round(float(v), 4) for n, v in zip(names, stage_avg)},
        'annotations_per_image': round(n_anns / max(1, args.steps * batch * world), 3)
        if stages & STAGE_GROW else None,
        # CifHr accumulation (the metric's "CifHr HBM GB/s"): CifHr.accumulated of the
        # reference API, the dense (K, H', W') map, pp_cifhr = cifhr_list_kernel +
        # cifhr_tile_kernel, timed on its own over `steps` launches on the same batch
        'roofline': {
            'bound': 'hbm', 'kernel': 'cifhr_list_kernel + cifhr_tile_kernel (pp_cifhr)',
            'achieved': round(dense_gbs, 1), 'peak': PEAK_HBM_GBS, 'unit': 'GB/s',
            'frac': round(dense_gbs / PEAK_HBM_GBS, 4), 'traffic': None,
            'algorithmic_bytes_per_launch': dense_bytes, 'ms_per_launch': round(dense_ms, 4),
        },
        # the decoder's own CifHr (inside `value`): the block-sparse map, written only where
        # splat boxes land; latency-bound per field, far below the dense byte count
        'roofline_decoder_cifhr': {
            'bound': 'hbm', 'kernel': 'cifhr_fused_kernel (CifHr + seed emission)',
            'achieved': round(achieved, 1), 'peak': PEAK_HBM_GBS, 'unit': 'GB/s',
            'frac': round(achieved / PEAK_HBM_GBS, 4),
            'algorithmic_bytes_per_launch': cifhr_bytes, 'traffic': None,
            # the same bytes counted in the 64-B lines they live in: the x / y / scale rows
            # of kept cells are 4-B gathers, a line per run of kept cells
            'line_granular_bytes_per_launch': sector_bytes,
            'written_block_frac': round(hr_tiles, 6),
            'us_per_image': round(1e3 * stage_avg[0] / batch, 4),
            'dense_equivalent_gbs': round(dense_bytes / (stage_avg[0] * 1e-3) / 1e9, 1),
        },
    }
    if world > 1:
        # the multi-GPU hand-over proves itself: every gathered step (the untimed one before
        # the clock and all timed ones) had each sender's record digest match on rank 0
        line['gather_verified'] = bool(gather['steps'] > 0 and
                                       gather['verified_steps'] == gather['steps'])
        line['ranks_seen'] = gather['ranks_seen']
        line['gather'] = {'steps': gather['steps'], 'verified_steps': gather['verified_steps'],
                          'full_record_steps': gather['full_record_steps'],
                          'bytes_per_step_rank0': gather['bytes']}
        # per rank: wall clock of the timed steps, device ms per step (first to last event of
        # a step; overlapped steps share the device), host ms per step blocked on the
        # step's records, host ms per step in the gather (rank 0: receiving and checking)
        line['per_rank'] = per_rank
    default_run = (args.workload in ('cfg3', 'cfg4') and args.generator == 'planted' and
                   args.mode == 'eval' and batch == WORKLOADS['cfg3']['batch'])
    if default_run:
        tr = committed_traffic()
        for key in ('roofline', 'roofline_decoder_cifhr'):
            if key in tr:
                line[key].update(tr[key])
        reconcile_trace(line['roofline'], dense_bytes)
        reconcile_trace(line['roofline_decoder_cifhr'], cifhr_bytes)
    if default_run and world == 1 and not args.no_predict:
        # the same planted batch in predict defaults (SURVEY.md §8d cfg3 names eval and
        # predict defaults; PREDICT_CONFIG: the CLI's predict thresholds, force-complete off)
        p_steps = max(3, args.steps // 2)
        p_el, p_stage, p_anns = timed_run(cif, caf, p_steps, 2,
                                          run_cfg=make_config(**PREDICT_CONFIG))
        log('predict done')
        line['predict'] = {
            'value': round(batch * p_steps / p_el, 1), 'unit': 'images/s',
            'ms_per_step': round(1e3 * p_el / p_steps, 4),
            'stage_ms': {n: round(float(v), 4) for n, v in zip(names, p_stage)},
            'annotations_per_image': round(p_anns / (p_steps * batch), 3),
        }
    if default_run and world == 1 and not args.no_uniform:
        # the same workload on the uniform generator (SURVEY.md §8d cfg3 names both):
        # dense random fields, ~400 annotations per image
        del cif, caf
        ucif, ucaf = synthetic.batch('uniform', batch, h, w, n_caf=len(skeleton))
        ucif, ucaf = torch.from_numpy(ucif).to(dev), torch.from_numpy(ucaf).to(dev)
        u_steps = max(3, args.steps // 2)
        u_el, u_stage, u_anns = timed_run(ucif, ucaf, u_steps, 2)
        log('uniform done')
        line['uniform'] = {
            'value': round(batch * u_steps / u_el, 1), 'unit': 'images/s',
            'ms_per_step': round(1e3 * u_el / u_steps, 4),
            'stage_ms': {n: round(float(v), 4) for n, v in zip(names, u_stage)},
            'annotations_per_image': round(u_anns / (u_steps * batch), 3),
        }
        # the dense CifHr map (pp_cifhr) on the uniform batch: ~15.5M pixel-visits per image
        # make it fold-bound, far from the write-bound planted case of `roofline`
        u_dense_ms = dense_cifhr_ms(ucif, cfg, stream, max(3, args.steps // 4), 1)
        u_gbs = dense_bytes / (u_dense_ms * 1e-3) / 1e9
        line['roofline_uniform'] = {
            'bound': 'hbm', 'kernel': 'cifhr_list_kernel + cifhr_tile_kernel (pp_cifhr), '
                                      'uniform generator',
            'achieved': round(u_gbs, 1), 'peak': PEAK_HBM_GBS, 'unit': 'GB/s',
            'frac': round(u_gbs / PEAK_HBM_GBS, 4), 'ms_per_launch': round(u_dense_ms, 4),
            'algorithmic_bytes_per_launch': dense_bytes,
            'decoder_cifhr_ms': round(float(u_stage[0]), 4),
        }
    if default_run and world == 1 and not args.no_multi:
        # multi-scale FieldConfigs (factory.py:153-180) on pp_decode_multi: the same people
        # seen by several heads; 'ms2' = stride 8 + 16 heads, 'ms10' = the reference's
        # 10-head hflip-pair layout (cif_hr.py:63-68)
        from openpifpaf_amd.decoder import FieldConfig
        from openpifpaf_amd.engine import HeadSet
        line['multi'] = {}
        px = (h - 1) * 8 + 1
        for name, n_img in (('ms2', batch), ('ms10', batch // 4)):
            per = [synthetic.multi_case(name, seed=i, h_px=px, w_px=px, n_people=wl['n_people'])
                   for i in range(n_img)]
            fields = [torch.from_numpy(np.stack([p[0][j] for p in per])).to(dev)
                      for j in range(len(per[0][0]))]
            heads = HeadSet(fields, FieldConfig(**per[0][1]))
            del per
            m_steps = max(3, args.steps // 2)
            m_el, m_stage, m_anns = timed_run(None, None, m_steps, 2, heads=heads)
            line['multi'][name] = {
                'value': round(n_img * m_steps / m_el, 1), 'unit': 'images/s',
                'images': n_img, 'image_px': px, 'heads': len(heads.cifs),
                'ms_per_step': round(1e3 * m_el / m_steps, 4),
                'stage_ms': {n: round(float(v), 4) for n, v in zip(names, m_stage)},
                'annotations_per_image': round(m_anns / (m_steps * n_img), 3),
            }
            del heads, fields
            log('multi {} done'.format(name))
    if default_run and world == 1 and not args.no_configs:
        # configs[1] (cfg2): batch-1 CifHr + seeds latency, host wall clock per call
        # (launch overhead + one synchronisation) and device time
        line['cfg2'] = {g: cfg2_latency(g, cfg, dev) for g in ('planted', 'uniform')}
        log('cfg2 done')
        # configs[4] (cfg5): 160x160, dense 44-CAF skeleton, 64 images per GPU
        w5 = WORKLOADS['cfg5']
        line['cfg5'] = {}
        for g in ('planted', 'uniform'):
            kw5 = ({'n_caf': len(constants.DENSE_DECODE_SKELETON)} if g == 'uniform' else
                   {'skeleton': constants.DENSE_DECODE_SKELETON, 'n_people': w5['n_people']})
            c5, a5 = synthetic.batch(g, w5['batch'], w5['h'], w5['w'], **kw5)
            c5, a5 = torch.from_numpy(c5).to(dev), torch.from_numpy(a5).to(dev)
            s5 = max(3, args.steps // (2 if g == 'planted' else 4))
            el5, st5, an5 = timed_run(c5, a5, s5, 1, skel=constants.DENSE_DECODE_SKELETON)
            line['cfg5'][g] = {
                'value': round(w5['batch'] * s5 / el5, 1), 'unit': 'images/s',
                'images': w5['batch'], 'field': '{}x{}'.format(w5['h'], w5['w']),
                'caf_fields': len(constants.DENSE_DECODE_SKELETON),
                'ms_per_step': round(1e3 * el5 / s5, 4),
                'stage_ms': {n: round(float(v), 4) for n, v in zip(names, st5)},
                'annotations_per_image': round(an5 / (s5 * w5['batch']), 3),
            }
            del c5, a5
            log('cfg5 {} done'.format(g))
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        uc = synthetic.batch('uniform', 64, h, w, n_caf=len(skeleton)) if default_run else None
        line['cpu_baseline'] = cpu_baseline(cif_h, caf_h, skeleton, cfg, args.cpu_seconds,
                                            *(uc or (None, None)))
    line['library'] = library_identity()
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def library_identity():
    """Which library the line measured: `src_sha` (openpifpaf_amd.build.source_digest of
    csrc/* and the header, the key profiles/<tag>_summary.json files are matched by), the
    sha256 of the loaded .so itself, its variant ('product' unless PP_LIB_VARIANT loaded a
    diagnostic or A/B build), and every PP_* environment variable this process saw.  The
    product library reads none of them (diagnostic builds read their stamp paths), and the
    Python pipeline's scheduling choices are constants (engine._B_FIRST ...).  `headline`
    is false when the line did not run the product library."""
    import hashlib
    from openpifpaf_amd import _lib
    from openpifpaf_amd.build import source_digest
    with open(_lib.LIB_PATH, 'rb') as f:
        so_sha = hashlib.sha256(f.read()).hexdigest()[:16]
    env = {k: v for k, v in sorted(os.environ.items()) if k.startswith('PP_')}
    variant = os.environ.get('PP_LIB_VARIANT') or 'product'
    return {'src_sha': source_digest(), 'so_sha256_16': so_sha,
            'so': os.path.relpath(_lib.LIB_PATH, REPO), 'variant': variant, 'pp_env': env,
            'headline': variant == 'product' and not env}


def cifhr_stage_bytes(cif, stride, v_th, seed_th=None, tile=64, block=8, lds_list=256):
    """Algorithmic HBM bytes of the decoder's CifHr stage (cifhr_fused_kernel: the
    block-sparse map and the seed emission) over a batch (n, K, 5, H, W): the confidence
    plane of every cell, the x / y / scale rows of passing cells, the splat records beyond
    the field's LDS-resident list written and read once (32 B each), the 8x8 blocks of the
    block-sparse map that splat boxes touch (256 B each, the same box arithmetic as
    splat_box in csrc/splat.hip), one u64 block mask per 64x64 tile, and per seed candidate
    (c > seed_th) its 16-B record written, read back with the CifHr block value and mask at
    its position, and the kept seed's 20 B written.  Returns (bytes, fraction of the map's
    blocks written, the same bytes with the x / y / scale gathers counted as the 64-B lines
    they touch)."""
    n, k, _, h, w = cif.shape
    hh, ww = (h - 1) * stride + 1, (w - 1) * stride + 1
    tiles_x = (-(-ww // 32) * 32 + tile - 1) // tile
    tiles_y = (hh + tile - 1) // tile
    c = cif[:, :, 0]
    keep = c > np.float32(v_th)
    per_field = keep.reshape(n * k, -1).sum(axis=1)
    img, fld, cy_i, cx_i = np.nonzero(keep)
    x = cif[img, fld, 1, cy_i, cx_i] * np.float32(stride)
    y = cif[img, fld, 2, cy_i, cx_i] * np.float32(stride)
    sg = (np.float32(0.5) * cif[img, fld, 4, cy_i, cx_i]) * np.float32(stride)
    sigma = np.where(np.isnan(sg), sg, np.maximum(np.float32(1.0), sg))

    def span(cen, size):
        lo = np.fmax(np.float32(0), np.fmin(np.float32(size - 1), cen - sigma))
        lo = np.nan_to_num(lo).astype(np.int64)
        hi = np.fmax((lo + 1).astype(np.float32), np.fmin(np.float32(size), (cen + sigma) + np.float32(1)))
        hi = np.nan_to_num(hi, nan=size).astype(np.int64)
        return lo // block, (hi - 1) // block

    bx0, bx1 = span(x, ww)
    by0, by1 = span(y, hh)
    touched = np.zeros((n, k, tiles_y * tile // block, tiles_x * tile // block), bool)
    for dy in range(int((by1 - by0).max(initial=0)) + 1):
        for dx in range(int((bx1 - bx0).max(initial=0)) + 1):
            m = (by0 + dy <= by1) & (bx0 + dx <= bx1)
            touched[img[m], fld[m], by0[m] + dy, bx0[m] + dx] = True
    n_blocks = int(touched.sum())
    overflow = int(np.maximum(per_field - lds_list, 0).sum())
    n_seed = int((c > np.float32(seed_th)).sum()) if seed_th is not None else 0
    seed_bytes = n_seed * (16 + 16 + 4 + 8 + 20)
    rest = (4 * n * k * h * w + 64 * overflow + n_blocks * 4 * block * block +
            8 * n * k * tiles_x * tiles_y + seed_bytes)
    # kept cells' rows at 64-B line granularity: distinct (plane row, 16-cell segment) pairs
    lines = len(np.unique(((img * k + fld) * h + cy_i) * ((w + 15) // 16) + cx_i // 16))
    return rest + 12 * len(img), n_blocks / touched.size, rest + 3 * 64 * lines


def dense_cifhr_ms(cif, cfg, stream, steps, warmup):
    """Average ms of one pp_cifhr launch (the dense CifHr.accumulated map of the whole
    resident batch) over `steps` back-to-back launches, HIP events on the launch stream."""
    import ctypes
    import torch
    from openpifpaf_amd import _device
    from openpifpaf_amd._lib import call, load
    lib = load()
    n, k, _, h, w = cif.shape
    hh, ww = (h - 1) * cfg.stride + 1, (w - 1) * cfg.stride + 1
    out = torch.empty((n, k, hh, int(lib.pp_cifhr_pitch(ww))), dtype=torch.float32,
                      device=cif.device)
    ws = torch.empty(int(lib.pp_cifhr_workspace_size(n, k, h, w)), dtype=torch.uint8,
                     device=cif.device)

    def launch():
        call('pp_cifhr', _device.ptr(cif), n, k, h, w, ctypes.byref(cfg), _device.ptr(out),
             _device.ptr(ws), ctypes.c_size_t(ws.numel()), _device.stream())

    for _ in range(max(1, warmup)):
        launch()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(stream)
    for _ in range(steps):
        launch()
    e1.record(stream)
    torch.cuda.synchronize()
    del out, ws
    return e0.elapsed_time(e1) / steps


# roofline key -> the kernels whose PMC bytes it reports (tools/prof_summary.py)
TRAFFIC_KERNELS = {'roofline': 'cifhr_list_kernel+cifhr_tile_kernel',
                   'roofline_decoder_cifhr': 'cifhr_fused_kernel'}


def committed_traffic():
    """HBM bytes per launch of the CifHr kernels from the committed PMC profile of this same
    workload and this same library (profiles/<tag>_summary.json, written by
    tools/prof_summary.py from the rocprofv3 FETCH_SIZE / WRITE_SIZE passes of
    tools/gpu_profile.sh; counters cannot be read from inside the timed process).  A
    profile counts only when its `src_sha` equals the running library's
    (openpifpaf_amd.build.source_digest); otherwise traffic is null and `traffic_stale`
    names the newest profile.  {roofline key: {traffic, traffic_source}}."""
    import glob
    from openpifpaf_amd.build import source_digest
    paths = sorted(glob.glob(os.path.join(REPO, 'profiles', 'r*_summary.json')))
    if not paths:
        return {}
    want = source_digest()
    summ, used = None, None
    for p in reversed(paths):
        with open(p) as f:
            s = json.load(f)
        if s.get('src_sha') == want:
            summ, used = s, p
            break
    out = {}
    for key, kernels in TRAFFIC_KERNELS.items():
        t = None if summ is None else summ.get('traffic_bytes', {}).get(kernels)
        if t is not None:
            out[key] = {'traffic': t, 'traffic_source': 'profiles/{} (src_sha {})'.format(
                os.path.basename(used), want)}
            # the same profile's kernel-trace average (rocprofv3 --kernel-trace, the
            # kernels' summed AverageNs in <tag>_kernel_stats.csv)
            avg = summ.get('avg_ns', {}).get(kernels)
            if avg:
                out[key]['trace_ms_per_launch'] = round(avg * 1e-6, 4)
        else:
            out[key] = {'traffic': None, 'traffic_stale': 'no committed profile of library '
                        '{} (newest: profiles/{})'.format(want, os.path.basename(paths[-1]))}
    return out


def reconcile_trace(roof, alg_bytes, tol=0.05):
    """Put the committed kernel trace's figure beside the live HIP-event one: `frac_events`
    (this run's events), `frac_trace` (algorithmic bytes over the trace average of the
    profile named in `traffic_source`).  When they differ by more than `tol`, `achieved` /
    `frac` report the lower one and `frac_source` says which; boxes differ by 10-20 %
    (DESIGN.md §4), so the headline never rests on the faster box alone."""
    ev_gbs = roof['achieved']
    roof['frac_events'] = roof['frac']
    trace_ms = roof.get('trace_ms_per_launch')
    if not trace_ms:
        roof['frac_source'] = 'events (no committed trace of this library)'
        return
    tr_gbs = alg_bytes / (trace_ms * 1e-3) / 1e9
    roof['frac_trace'] = round(tr_gbs / roof['peak'], 4)
    if abs(tr_gbs - ev_gbs) > tol * max(tr_gbs, ev_gbs) and tr_gbs < ev_gbs:
        roof['achieved'] = round(tr_gbs, 1)
        roof['frac'] = roof['frac_trace']
        roof['frac_source'] = 'trace (lower than events by more than {:.0%})'.format(tol)
    else:
        roof['frac_source'] = 'events (within {:.0%} of the trace, or lower)'.format(tol)


def cfg2_latency(gen, cfg, dev, calls=200):
    """BASELINE.json configs[1]: one 80x80 image, CifHr + seeds only (pp_decode_stages with
    stages 1 | 2).  Host: median wall clock of launch + synchronise per call; device: HIP
    events over `calls` back-to-back calls."""
    import torch
    from openpifpaf_amd import synthetic
    from openpifpaf_amd.engine import STAGE_CIFHR, STAGE_SEEDS, DecodeEngine
    from openpifpaf_amd import constants
    cif, caf = synthetic.batch(gen, 1, 80, 80)
    cif, caf = torch.from_numpy(cif).to(dev), torch.from_numpy(caf).to(dev)
    eng = DecodeEngine()
    skel = constants.COCO_PERSON_SKELETON

    def run():
        eng.launch(cif, caf, skel, cfg, stages=STAGE_CIFHR | STAGE_SEEDS)

    for _ in range(5):
        run()
    torch.cuda.synchronize()
    host = []
    for _ in range(calls):
        t0 = time.perf_counter()
        run()
        torch.cuda.synchronize()
        host.append(time.perf_counter() - t0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(calls):
        run()
    e1.record()
    torch.cuda.synchronize()
    return {'us_per_call_host': round(1e6 * float(np.median(host)), 2),
            'us_per_call_device': round(1e3 * e0.elapsed_time(e1) / calls, 2),
            'calls': calls}


def cpu_share():
    """(threads to use, how they were counted): the CPUs this process may run on
    (sched_getaffinity), capped by the cgroup's CPU quota where one is set (cpu.max, as on
    the GPU box, whose affinity mask shows the whole machine)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:
        with open('/sys/fs/cgroup/cpu.max') as f:
            q, period = f.read().split()[:2]
        if q != 'max':
            quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        pass
    cores = min(aff, quota) if quota else aff
    return cores, {'affinity_cpus': aff, 'cgroup_cpu_quota': quota}


def cpu_baseline(cif, caf, skeleton, cfg, budget_s, ucif=None, ucaf=None):
    """The oracle (C restatement of the reference decoder) on the host cores, over a bounded
    sample of the same images: one thread, then one thread per CPU of this job's share
    (cpu_share(); ctypes releases the GIL for the C decode; the oracle has no global state),
    cycling over the batch; then the uniform batch on every thread.  The reference's own
    Cython decoder cannot travel to the GPU box; profiles/cpu_ratio.json (tools/cpu_ratio.py,
    measured in the build container on the same generators) gives the reference/oracle time
    ratio per generator, so `reference_equivalent` = oracle rate / ratio."""
    import concurrent.futures
    sys.path.insert(0, os.path.join(REPO, 'oracle'))
    import oracle  # pylint: disable=import-outside-toplevel
    oracle.lib()

    def worker(c, a, first, budget):
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < budget:
            i = (first + n) % len(c)
            oracle.decode(c[i], a[i], skeleton, cfg)
            n += 1
        return n, time.perf_counter() - t0

    def all_threads(c, a, budget):
        with concurrent.futures.ThreadPoolExecutor(cores) as ex:
            res = list(ex.map(lambda t: worker(c, a, 17 * t, budget), range(cores)))
        return sum(n for n, _ in res), max(dt for _, dt in res)

    n1, dt1 = worker(cif, caf, 0, budget_s / 3)
    one = n1 / dt1
    cores, share = cpu_share()
    na, dta = all_threads(cif, caf, budget_s / 3)
    allc = na / dta
    out = {'value': round(allc, 2), 'unit': 'images/s', 'cores': cores, 'kind': 'port',
           'single_core': round(one, 2),
           'sample': '{} single-image decodes on one core in {:.1f} s, then {} on {} threads in '
                     '{:.1f} s, cycling over the planted batch; oracle/pp_oracle.c'.format(
                         n1, dt1, na, cores, dta),
           'cores_from': share, 'host_cpu_count': os.cpu_count()}
    try:
        with open(os.path.join(REPO, 'profiles', 'cpu_ratio.json')) as f:
            ratios = json.load(f)['cases']
    except (OSError, KeyError, ValueError):
        ratios = {}
    if 'planted' in ratios:
        r = ratios['planted']
        out['reference_over_oracle_time'] = r['ratio']
        out['reference_equivalent'] = {
            'single_core': round(one / r['ratio'], 2),
            'all_cores': round(allc / r['ratio'], 2),
            'source': 'profiles/cpu_ratio.json (reference vs oracle total time over {} planted '
                      '80x80 eval images, one thread, build container)'.format(r['images'])}
    # the build's own C++ twin of the decode (pp_decode_batch_cpu, csrc/decode_cpu.hip:
    # bit-exact with the device and the reference, SURVEY.md §8d's CPU comparator) on the
    # same threads, whole chunks of the planted batch per call
    from openpifpaf_amd import stages_cpu
    chunk = max(4 * cores, 16)
    nt, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s / 4:
        i = (nt % len(cif))
        c, a = cif[i:i + chunk], caf[i:i + chunk]
        stages_cpu.decode_batch(c, a, skeleton, cfg, n_threads=cores)
        nt += len(c)
    dtt = time.perf_counter() - t0
    out['twin'] = {'value': round(nt / dtt, 2), 'unit': 'images/s', 'cores': cores,
                   'kind': 'twin',
                   'sample': '{} planted decodes by pp_decode_batch_cpu on {} threads in '
                             '{:.1f} s'.format(nt, cores, dtt)}
    if ucif is not None:
        nu, dtu = all_threads(ucif, ucaf, budget_s / 3)
        out['uniform'] = {'value': round(nu / dtu, 2), 'unit': 'images/s', 'cores': cores,
                          'sample': '{} uniform decodes on {} threads in {:.1f} s'.format(
                              nu, cores, dtu)}
        if 'uniform' in ratios:
            out['uniform']['reference_over_oracle_time'] = ratios['uniform']['ratio']
            out['uniform']['reference_equivalent'] = round(
                nu / dtu / ratios['uniform']['ratio'], 2)
    return out


if __name__ == '__main__':
    main()
