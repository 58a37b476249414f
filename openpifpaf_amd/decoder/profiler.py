"""--profile-decoder wrappers (decoder/profiler.py, decoder/profiler_autograd.py).

Profiler: cProfile around each call, stats sorted by tottime printed and dumped to
`out_name`.  ProfilerAutograd: a torch.profiler trace (CPU + HIP activity) around each
call, printed as key averages and exported as numbered chrome traces.
"""
import cProfile
import io
import logging
import pstats

import torch

LOG = logging.getLogger(__name__)


class Profiler:
    def __init__(self, function_to_profile, *, profile=None, out_name=None):
        self.function_to_profile = function_to_profile
        self.profile = cProfile.Profile() if profile is None else profile
        self.out_name = out_name

    def __call__(self, *args, **kwargs):
        self.profile.enable()
        try:
            return self.function_to_profile(*args, **kwargs)
        finally:
            self.profile.disable()
            out = io.StringIO()
            stats = pstats.Stats(self.profile, stream=out).sort_stats('tottime')
            stats.print_stats()
            if self.out_name:
                LOG.info('writing profile file %s', self.out_name)
                stats.dump_stats(self.out_name)
            print(out.getvalue())


class ProfilerAutograd:
    trace_counter = 0

    def __init__(self, function_to_profile, *, device, out_name=None):
        self.function_to_profile = function_to_profile
        self.device = device
        self.out_name = out_name or 'pytorch_chrome_trace.json'

    def __call__(self, *args, **kwargs):
        acts = [torch.profiler.ProfilerActivity.CPU]
        if str(self.device).startswith('cuda'):
            acts.append(torch.profiler.ProfilerActivity.CUDA)
        with torch.profiler.profile(activities=acts) as prof:
            result = self.function_to_profile(*args, **kwargs)
        print(prof.key_averages())
        type(self).trace_counter += 1
        name = '{}.{}.json'.format(self.out_name.replace('.json', '').replace('.prof', ''),
                                   self.trace_counter)
        LOG.info('writing trace file %s', name)
        prof.export_chrome_trace(name)
        return result
