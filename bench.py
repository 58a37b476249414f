"""Benchmark: batched CIF/CAF decode on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload cfg3|cfg2|cfg5]
                    [--generator planted|uniform] [--mode eval|predict]

One step = one full decode (CifHr -> seeds -> CafScored -> seed loop / grow ->
force-complete -> NMS) of the rank's resident batch of synthetic fields, plus the packing
of its annotation records into pinned host memory (steps are pipelined two deep: step k + 1
is enqueued before step k's records are waited for); for N > 1 also the
RCCL all-gather of every rank's records to rank 0 (weak scaling: each rank owns its own
batch, no data-path collective).  Inputs are generated once and stay in HBM.

Rank 0 prints ONE JSON line.  `roofline` is the CifHr accumulation of the metric: the
dense CifHr.accumulated map (pp_cifhr) of the same resident batch, timed with HIP events
on the launch stream; algorithmic bytes = 4*K*(5*H*W + H'*W') per image
over its launch time.  `roofline_decoder_cifhr` is the decoder's own block-sparse CifHr
stage inside `value` (its bytes: bench.cifhr_stage_bytes).
`cpu_baseline` is the oracle (oracle/pp_oracle.c, C restatement of the reference decoder)
on one host core over a bounded sample of the same workload.
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
    # configs[1]: batch 1, CifHr + seeds only
    'cfg2': dict(h=80, w=80, batch=1, skeleton='coco', n_people=8, stages=3),
    # configs[4]: 160x160, dense 44-CAF skeleton, 64 images per GPU
    'cfg5': dict(h=160, w=160, batch=64, skeleton='dense', n_people=16),
}
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=20)
    p.add_argument('--warmup', type=int, default=3)
    p.add_argument('--workload', default='cfg3', choices=sorted(WORKLOADS))
    p.add_argument('--generator', default='planted', choices=('planted', 'uniform'))
    p.add_argument('--mode', default='eval', choices=('eval', 'predict'))
    p.add_argument('--batch', type=int, default=None, help='images per GPU (override)')
    p.add_argument('--cpu-seconds', type=float, default=12.0,
                   help='budget of the oracle CPU baseline sample (rank 0, N=1)')
    p.add_argument('--no-cpu-baseline', action='store_true')
    p.add_argument('--no-uniform', action='store_true',
                   help='skip the uniform-generator line added to the default run')
    p.add_argument('--no-multi', action='store_true',
                   help='skip the multi-scale (pp_decode_multi) lines added to the default run')
    p.add_argument('--stage-breakdown', action='store_true',
                   help='one library call per stage (per-stage times)')
    return p.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        dist.init_process_group('nccl', device_id=torch.device('cuda', local_rank))
    torch.cuda.set_device(local_rank)
    dev = torch.device('cuda', local_rank)

    from openpifpaf_amd import build as ppbuild
    ppbuild.build(verbose=False)
    from openpifpaf_amd import constants, synthetic
    from openpifpaf_amd.distributed import gather_records
    from openpifpaf_amd._abi import EVAL_CONFIG, PREDICT_CONFIG, make_config
    from openpifpaf_amd.engine import (STAGE_CAF, STAGE_CIFHR, STAGE_GROW, STAGE_SEEDS,
                                       DecodeEngine)

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
    # default: CifHr alone (its events give the roofline), then the other stages in one
    # call; --stage-breakdown: one call per stage
    groups = ((STAGE_CIFHR, STAGE_SEEDS, STAGE_CAF, STAGE_GROW) if args.stage_breakdown else
              (STAGE_CIFHR, STAGE_SEEDS | STAGE_CAF | STAGE_GROW))
    names = (('cifhr', 'seeds', 'caf_scored', 'grow_nms') if args.stage_breakdown else
             ('cifhr', 'seeds+caf+grow+nms'))
    # two event sets: with the two-deep pipeline, step k's events are read after step k + 1
    # has recorded its own
    ev_sets = [[torch.cuda.Event(enable_timing=True) for _ in range(len(groups) + 1)]
               for _ in range(2)]

    def timed_run(cif, caf, steps, warmup, heads=None):
        """warmup + `steps` timed decode steps of one resident batch (cif / caf, or a
        multi-scale HeadSet): (elapsed s over all ranks, per-group event ms per step,
        annotations decoded)."""
        stage_ms = np.zeros(len(groups))

        def step(timed, k=0):
            """Enqueue one decode and its record fetch; returns (buffers, (PendingRecords,
            its event set))."""
            ev = ev_sets[k % 2]
            b = None
            for si, bits in enumerate(groups):
                if timed:
                    ev[si].record(stream)
                if stages & bits and heads is not None:
                    b = eng.launch_multi(heads, skeleton, cfg, stages=stages & bits)
                elif stages & bits:
                    b = eng.launch(cif, caf, skeleton, cfg, stages=stages & bits)
            if timed:
                ev[len(groups)].record(stream)
            # packed records -> pinned host memory, enqueued behind the decode
            return b, ((eng.fetch_async(b) if stages & STAGE_GROW else None), ev)

        def finish(step_out, timed):
            """Wait for one step's records (and, for N > 1, gather them to rank 0)."""
            pending, ev = step_out
            n_recs = 0
            if pending is None:
                torch.cuda.synchronize()
            else:
                recs, offsets = pending.result()
                if world > 1:
                    recs, _ = gather_records(recs, offsets, dist, dev)
                n_recs = len(recs)
            if timed:
                ev[len(groups)].synchronize()
                for si in range(len(groups)):
                    stage_ms[si] += ev[si].elapsed_time(ev[si + 1])
            return n_recs

        for _ in range(warmup):
            b, p = step(False)
            finish(p, False)
        status = b.status.cpu().numpy()
        if status.any():
            raise SystemExit('decode status flags set: {}'.format(status[status != 0][:8]))
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n_anns = 0
        # two-deep pipeline: step k + 1 is enqueued before step k's records are waited for
        # (decode outputs are double-buffered, engine.DecodeBuffers), so the host's record
        # handling and next launches overlap the device work; every step's records are on
        # the host before the clock stops
        pending = None
        for k in range(steps):
            b, p = step(True, k)
            if pending is not None:
                n_anns += finish(pending, True)
            pending = p
        n_anns += finish(pending, True)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        return elapsed, stage_ms / steps, n_anns

    elapsed, stage_avg, n_anns = timed_run(cif, caf, args.steps, args.warmup)

    images = batch * world * args.steps
    value = images / elapsed
    ms_step = 1e3 * elapsed / args.steps
    hh, ww = (h - 1) * 8 + 1, (w - 1) * 8 + 1
    cifhr_bytes, hr_tiles = cifhr_stage_bytes(cif_h, 8, cfg.cif_threshold)
    achieved = cifhr_bytes / (stage_avg[0] * 1e-3) / 1e9
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
            'parallelism': 'image-sharded dp{} (RCCL all-gather of annotation records)'.format(
                world) if world > 1 else 'single GPU',
        },
        'stage_ms': {n: round(float(v), 4) for n, v in zip(names, stage_avg)},
        'annotations_per_image': round(n_anns / max(1, args.steps * batch * world), 3)
        if stages & STAGE_GROW else None,
        # CifHr accumulation (the metric's "CifHr HBM GB/s"): CifHr.accumulated of the
        # reference API, the dense (K, H', W') map, pp_cifhr = cifhr_splats_kernel +
        # cifhr_tile_kernel, timed on its own over `steps` launches on the same batch
        'roofline': {
            'bound': 'hbm', 'kernel': 'cifhr_splats_kernel + cifhr_tile_kernel (pp_cifhr)',
            'achieved': round(dense_gbs, 1), 'peak': PEAK_HBM_GBS, 'unit': 'GB/s',
            'frac': round(dense_gbs / PEAK_HBM_GBS, 4), 'traffic': None,
            'algorithmic_bytes_per_launch': dense_bytes, 'ms_per_launch': round(dense_ms, 4),
        },
        # the decoder's own CifHr (inside `value`): the block-sparse map, written only where
        # splat boxes land; latency-bound per field, far below the dense byte count
        'roofline_decoder_cifhr': {
            'bound': 'hbm', 'kernel': 'cifhr_sparse_kernel',
            'achieved': round(achieved, 1), 'peak': PEAK_HBM_GBS, 'unit': 'GB/s',
            'frac': round(achieved / PEAK_HBM_GBS, 4),
            'algorithmic_bytes_per_launch': cifhr_bytes, 'traffic': None,
            'written_block_frac': round(hr_tiles, 6),
            'us_per_image': round(1e3 * stage_avg[0] / batch, 4),
            'dense_equivalent_gbs': round(dense_bytes / (stage_avg[0] * 1e-3) / 1e9, 1),
        },
    }
    default_run = (args.workload == 'cfg3' and args.generator == 'planted' and
                   args.mode == 'eval' and batch == WORKLOADS['cfg3']['batch'])
    if default_run:
        tr = committed_traffic()
        for key in ('roofline', 'roofline_decoder_cifhr'):
            if key in tr:
                line[key].update(tr[key])
    if default_run and world == 1 and not args.no_uniform:
        # the same workload on the uniform generator (SURVEY.md §8d cfg3 names both):
        # dense random fields, ~400 annotations per image
        del cif, caf
        ucif, ucaf = synthetic.batch('uniform', batch, h, w, n_caf=len(skeleton))
        ucif, ucaf = torch.from_numpy(ucif).to(dev), torch.from_numpy(ucaf).to(dev)
        u_steps = max(3, args.steps // 2)
        u_el, u_stage, u_anns = timed_run(ucif, ucaf, u_steps, 2)
        line['uniform'] = {
            'value': round(batch * u_steps / u_el, 1), 'unit': 'images/s',
            'ms_per_step': round(1e3 * u_el / u_steps, 4),
            'stage_ms': {n: round(float(v), 4) for n, v in zip(names, u_stage)},
            'annotations_per_image': round(u_anns / (u_steps * batch), 3),
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
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line['cpu_baseline'] = cpu_baseline(cif_h, caf_h, skeleton, cfg, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cifhr_stage_bytes(cif, stride, v_th, tile=64, block=8, lds_list=256):
    """Algorithmic HBM bytes of the decoder's CifHr stage (cifhr_sparse_kernel) over a
    batch (n, K, 5, H, W): the confidence plane of every cell, the x / y / scale rows of
    passing cells, the splat records beyond the field's LDS-resident list written and read
    once (32 B each), the 8x8 blocks of the block-sparse map that splat boxes touch (256 B
    each, the same box arithmetic as splat_box in csrc/splat.hip) and one u64 block mask per
    64x64 tile.  Returns (bytes, fraction of the map's blocks written)."""
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
    nbytes = (4 * n * k * h * w + 12 * len(img) + 64 * overflow +
              n_blocks * 4 * block * block + 8 * n * k * tiles_x * tiles_y)
    return nbytes, n_blocks / touched.size


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
TRAFFIC_KERNELS = {'roofline': 'cifhr_splats_kernel+cifhr_tile_kernel',
                   'roofline_decoder_cifhr': 'cifhr_sparse_kernel'}


def committed_traffic():
    """HBM bytes per launch of the CifHr kernels from the newest committed PMC profile of
    this same workload (profiles/<tag>_summary.json, written by tools/prof_summary.py from
    the rocprofv3 FETCH_SIZE / WRITE_SIZE passes of tools/gpu_profile.sh; counters cannot
    be read from inside the timed process).  {roofline key: {traffic, traffic_source}}."""
    import glob
    paths = sorted(glob.glob(os.path.join(REPO, 'profiles', 'r*_summary.json')))
    if not paths:
        return {}
    with open(paths[-1]) as f:
        summ = json.load(f)
    out = {}
    for key, kernels in TRAFFIC_KERNELS.items():
        t = summ.get('traffic_bytes', {}).get(kernels)
        if t is not None:
            out[key] = {'traffic': t, 'traffic_source': 'profiles/' + os.path.basename(paths[-1])}
    return out


def cpu_baseline(cif, caf, skeleton, cfg, budget_s):
    """Oracle (C restatement of the reference decoder) on one core, bounded sample."""
    sys.path.insert(0, os.path.join(REPO, 'oracle'))
    import oracle  # pylint: disable=import-outside-toplevel
    oracle.lib()
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        i = n % len(cif)
        oracle.decode(cif[i], caf[i], skeleton, cfg)
        n += 1
    dt = time.perf_counter() - t0
    return {'value': round(n / dt, 2), 'unit': 'images/s', 'cores': 1, 'kind': 'port',
            'sample': '{} single-image decodes (cycling over the first {} images of the '
                      'batch) in {:.1f} s on one host core; oracle/pp_oracle.c'.format(
                          n, min(n, len(cif)), dt),
            'host_cpu_count': os.cpu_count()}


if __name__ == '__main__':
    main()
