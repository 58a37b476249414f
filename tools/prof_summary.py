"""Summarise a tools/gpu_profile.sh run into profiles/<tag>_*.

    python tools/prof_summary.py r01

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats, verbatim),
profiles/<tag>_counters.csv (per kernel: launches, mean FETCH_SIZE / WRITE_SIZE bytes per
launch from the PMC passes), profiles/<tag>_calibration.csv (counter bytes / true bytes for
the calibration kernels) and profiles/<tag>_summary.json (per CifHr kernel set: duration
and corrected HBM traffic per launch, as bench.py's roofline objects report them).
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# kernel sets whose HBM bytes per launch the bench's roofline objects report
# (the dense map's phase 1 is cifhr_list_kernel from round 3 on, cifhr_splats_kernel before;
# at 256 images the decoder does not use cifhr_list_kernel, so in the cfg3 bench it is the
# dense map's alone)
KERNEL_SETS = (('cifhr_list_kernel', 'cifhr_tile_kernel'), ('cifhr_sparse_kernel',),
               ('cifhr_fused_kernel',))
CALIB_BYTES = 1 << 30


def short(name):
    """Kernel name without return type, namespace, template and parameter lists (the
    caf_bucketed_kernel<false> / <true> stages therefore share one row)."""
    name = name.split('(')[0]
    for pre in ('void ', 'pp::'):
        name = name.replace(pre, '')
    return name.split('<')[0].strip()


def counters(path):
    """kernel -> list of counter bytes per dispatch (rocprofv3 reports KB)."""
    per = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            per[short(row['Kernel_Name'])].append(float(row['Counter_Value']) * 1024.0)
    return per


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else 'r01'
    src = os.path.join(REPO, 'gpurun_out', 'prof_' + tag)
    dst = os.path.join(REPO, 'profiles')
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, 'kt', 'run_kernel_stats.csv'),
                os.path.join(dst, tag + '_kernel_stats.csv'))
    stats = {}
    with open(os.path.join(src, 'kt', 'run_kernel_stats.csv')) as f:
        for row in csv.DictReader(f):
            stats[short(row['Name'])] = (int(row['Calls']), float(row['AverageNs']))

    fetch = counters(os.path.join(src, 'pmc_FETCH_SIZE', 'run_counter_collection.csv'))
    write = counters(os.path.join(src, 'pmc_WRITE_SIZE', 'run_counter_collection.csv'))
    with open(os.path.join(dst, tag + '_counters.csv'), 'w', newline='') as f:
        w = csv.writer(f)
        w.writerow(['kernel', 'launches', 'avg_ns', 'fetch_bytes_per_launch',
                    'write_bytes_per_launch'])
        for k in sorted(set(fetch) | set(write)):
            fl, wl = fetch.get(k, []), write.get(k, [])
            w.writerow([k, len(fl), round(stats.get(k, (0, 0.0))[1], 1),
                        round(sum(fl) / max(1, len(fl))), round(sum(wl) / max(1, len(wl)))])

    calib = {}
    cf = counters(os.path.join(src, 'calib_FETCH_SIZE', 'run_counter_collection.csv'))
    cw = counters(os.path.join(src, 'calib_WRITE_SIZE', 'run_counter_collection.csv'))
    with open(os.path.join(dst, tag + '_calibration.csv'), 'w', newline='') as f:
        w = csv.writer(f)
        w.writerow(['kernel', 'true_bytes', 'counter', 'counter_bytes_mean', 'ratio'])
        for k, per, cname in (('read4', cf, 'FETCH_SIZE'), ('read16', cf, 'FETCH_SIZE'),
                              ('write4', cw, 'WRITE_SIZE'), ('write16', cw, 'WRITE_SIZE')):
            vals = per.get(k, [])
            mean = sum(vals) / max(1, len(vals))
            calib[k] = mean / CALIB_BYTES
            w.writerow([k, CALIB_BYTES, cname, round(mean), round(calib[k], 4)])

    # per-kernel correction by the calibrated ratio of the access width each one streams
    # with (tools/calib_counters.hip): 4 B field reads, 16 B nontemporal dense-map stores,
    # 4 B block stores of the sparse map
    read_width = {'cifhr_splats_kernel': 'read4', 'cifhr_list_kernel': 'read4', 'cifhr_tile_kernel': 'read16',
                  'cifhr_sparse_kernel': 'read4', 'cifhr_fused_kernel': 'read4'}
    write_width = {'cifhr_splats_kernel': 'write16', 'cifhr_list_kernel': 'write16', 'cifhr_tile_kernel': 'write16',
                   'cifhr_sparse_kernel': 'write4', 'cifhr_fused_kernel': 'write4'}
    sha_path = os.path.join(src, 'src_sha.txt')
    summary = {
        'tag': tag,
        # the library the profile measured (openpifpaf_amd.build.source_digest on the box)
        'src_sha': open(sha_path).read().strip() if os.path.exists(sha_path) else None,
        'fetch_ratio_16B': round(calib.get('read16', 0.0), 4),
        'fetch_ratio_4B': round(calib.get('read4', 0.0), 4),
        'write_ratio_16B': round(calib.get('write16', 0.0), 4),
        'write_ratio_4B': round(calib.get('write4', 0.0), 4),
        'avg_ns': {}, 'fetch_bytes_raw': {}, 'write_bytes_raw': {}, 'traffic_bytes': {},
    }
    for ks in KERNEL_SETS:
        if not all(k in fetch and k in write and k in stats for k in ks):
            continue
        name = '+'.join(ks)
        f_raw = sum(sum(fetch[k]) / len(fetch[k]) for k in ks)
        w_raw = sum(sum(write[k]) / len(write[k]) for k in ks)
        traffic = 0.0
        for k in ks:
            traffic += (sum(fetch[k]) / len(fetch[k])) / (calib.get(read_width[k]) or 1.0)
            traffic += (sum(write[k]) / len(write[k])) / (calib.get(write_width[k]) or 1.0)
        summary['avg_ns'][name] = round(sum(stats[k][1] for k in ks), 1)
        summary['fetch_bytes_raw'][name] = round(f_raw)
        summary['write_bytes_raw'][name] = round(w_raw)
        summary['traffic_bytes'][name] = round(traffic)
    with open(os.path.join(dst, tag + '_summary.json'), 'w') as f:
        json.dump(summary, f, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == '__main__':
    main()
