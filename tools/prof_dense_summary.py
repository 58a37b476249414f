"""Summarise a tools/gpu_profile_dense.sh run into profiles/<tag>_dense_*.

    python tools/prof_dense_summary.py r03a

Copies each workload's rocprofv3 --stats table verbatim (profiles/<tag>_dense_<name>.csv)
and writes profiles/<tag>_dense_summary.json: per workload the bench line's value,
ms_per_step, stage_ms and annotations per image, plus the per-kernel average durations.
"""
import csv
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    name = name.split('(')[0]
    for pre in ('void ', 'pp::'):
        name = name.replace(pre, '')
    return name.strip()


def main():
    tag = sys.argv[1]
    src = os.path.join(REPO, 'gpurun_out', 'profd_' + tag)
    dst = os.path.join(REPO, 'profiles')
    out = {}
    for name in sorted(os.listdir(src)):
        stats = os.path.join(src, name, 'run_kernel_stats.csv')
        if not os.path.isfile(stats):
            continue
        shutil.copy(stats, os.path.join(dst, '{}_dense_{}.csv'.format(tag, name)))
        with open(os.path.join(src, name + '_bench.json')) as f:
            line = json.load(f)
        kernels = {}
        with open(stats) as f:
            for row in csv.DictReader(f):
                if row['Name'].startswith('at::') or 'rocclr' in row['Name']:
                    continue
                kernels[short(row['Name'])] = {'calls': int(row['Calls']),
                                               'avg_us': round(float(row['AverageNs']) / 1e3, 1)}
        out[name] = {'value': line['value'], 'ms_per_step': line['ms_per_step'],
                     'stage_ms': line['stage_ms'],
                     'annotations_per_image': line['annotations_per_image'],
                     'workload': line['config']['workload'], 'data': line['data'],
                     'kernels': kernels}
    with open(os.path.join(dst, tag + '_dense_summary.json'), 'w') as f:
        json.dump(out, f, indent=1)
    print('wrote', os.path.join(dst, tag + '_dense_summary.json'))


if __name__ == '__main__':
    main()
