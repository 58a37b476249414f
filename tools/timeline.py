"""Per-step kernel timeline of an overlapped bench run from a rocprofv3 kernel trace.

    python tools/timeline.py gpurun_out/<dir>/run_kernel_trace.csv [first_step] [n_steps]

Steps are delimited by the decoder's CifHr kernel launches (one per step); prints each
kernel's start / end in microseconds relative to its step's CifHr start, with its queue.
"""
import csv
import sys


def short(name):
    name = name.split('(')[0]
    for pre in ('void ', 'pp::'):
        name = name.replace(pre, '')
    return name.strip()[:40]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    first = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    ks = sorted(((int(r['Start_Timestamp']), int(r['End_Timestamp']), short(r['Kernel_Name']),
                  r.get('Queue_Id', r.get('Stream_Id', '?'))) for r in rows))
    marks = [s for s, _, k, _ in ks if k.startswith('cifhr_fused') or k.startswith('cifhr_sparse')]
    if len(marks) < first + n + 1:
        first = max(0, len(marks) - n - 1)
    t0 = marks[first]
    t1 = marks[min(len(marks) - 1, first + n)]
    print('steps {}..{}: {:.1f} us per step'.format(first, first + n, (t1 - t0) / 1e3 / n))
    for s, e, k, q in ks:
        if s < t0 - 2_000_000 or s > t1:
            continue
        print('{:9.1f} {:9.1f} {:8.1f}  q{:>3}  {}'.format((s - t0) / 1e3, (e - t0) / 1e3,
                                                        (e - s) / 1e3, q, k))


if __name__ == '__main__':
    main()
