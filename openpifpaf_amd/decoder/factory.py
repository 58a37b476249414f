"""Decoder configuration and construction (decoder/factory.py:17-213).

cli()/configure() are the reference's: they write the same CLASS ATTRIBUTES, which the
device decoder reads at call time.  factory_decode() accepts the network's head nets or metas
(duck-typed) and builds a CifCaf (single-scale, dense connections, multi-scale with or
without hflip) or a CifDet, as the reference does.
"""
import logging

from .caf_scored import CafScored
from .cif_hr import CifHr
from .cif_seeds import CifSeeds
from .field_config import FieldConfig
from .generator.cifcaf import CifCaf
from .generator.cifdet import CifDet
from .profiler import Profiler, ProfilerAutograd
from . import nms

LOG = logging.getLogger(__name__)


def cli(parser, *, force_complete_pose=True, seed_threshold=0.2, instance_threshold=0.0,
        keypoint_threshold=None, workers=None):
    group = parser.add_argument_group('decoder configuration')
    group.add_argument('--seed-threshold', default=seed_threshold, type=float,
                       help='minimum threshold for seeds')
    group.add_argument('--instance-threshold', type=float, default=instance_threshold,
                       help='filter instances by score')
    group.add_argument('--keypoint-threshold', type=float, default=keypoint_threshold,
                       help='filter keypoints by score')
    group.add_argument('--decoder-workers', default=workers, type=int,
                       help='number of workers for pose decoding (ignored: device decode)')
    group.add_argument('--dense-connections', default=False, action='store_true',
                       help='use dense connections')
    group.add_argument('--dense-coupling', default=0.01, type=float, help='dense coupling')
    group.add_argument('--caf-seeds', default=False, action='store_true',
                       help='[experimental]')
    if force_complete_pose:
        group.add_argument('--no-force-complete-pose', dest='force_complete_pose',
                           default=True, action='store_false')
    else:
        group.add_argument('--force-complete-pose', dest='force_complete_pose',
                           default=False, action='store_true')
    group.add_argument('--profile-decoder', nargs='?', const='profile_decoder.prof',
                       default=None, help='specify out .prof file or nothing for default')

    group = parser.add_argument_group('CifCaf decoders')
    group.add_argument('--cif-th', default=CifHr.v_threshold, type=float, help='cif threshold')
    group.add_argument('--caf-th', default=CafScored.default_score_th, type=float,
                       help='caf threshold')
    group.add_argument('--connection-method', default=CifCaf.connection_method,
                       choices=('max', 'blend'), help='connection method to use, max is faster')
    group.add_argument('--greedy', default=False, action='store_true', help='greedy decoding')


def configure(args):
    if args.keypoint_threshold is None:
        args.keypoint_threshold = 0.001 if not args.force_complete_pose else 0.0
    if args.force_complete_pose:
        assert args.keypoint_threshold == 0.0
    assert args.seed_threshold >= args.keypoint_threshold

    CifHr.v_threshold = args.cif_th
    CifSeeds.threshold = args.seed_threshold
    CafScored.default_score_th = args.caf_th
    CifCaf.force_complete = args.force_complete_pose
    CifCaf.keypoint_threshold = args.keypoint_threshold
    CifCaf.greedy = args.greedy
    CifCaf.connection_method = args.connection_method
    nms.Detection.instance_threshold = args.instance_threshold
    nms.Keypoints.instance_threshold = args.instance_threshold
    nms.Keypoints.keypoint_threshold = args.keypoint_threshold

    # decoder workers (factory.py:93-98): the device decode ignores the pool, the default is
    # still written back for callers that read it
    if args.decoder_workers is None and getattr(args, 'batch_size', 1) > 1 and \
            not getattr(args, 'debug', False):
        args.decoder_workers = args.batch_size


def factory_from_args(args, model):
    configure(args)
    decode = factory_decode(model.head_nets,
                            basenet_stride=model.base_net.stride,
                            dense_coupling=args.dense_coupling,
                            dense_connections=args.dense_connections,
                            caf_seeds=args.caf_seeds,
                            multi_scale=getattr(args, 'multi_scale', False),
                            multi_scale_hflip=getattr(args, 'multi_scale_hflip', True),
                            worker_pool=args.decoder_workers)
    if args.profile_decoder is not None:  # factory.py:113-117
        decode.__class__.__call__ = Profiler(decode.__call__, out_name=args.profile_decoder)
        decode.fields_batch = ProfilerAutograd(decode.fields_batch,
                                               device=getattr(args, 'device', 'cuda'),
                                               out_name=args.profile_decoder)
        # batch() runs the network through _heads (batch-major, no per-image split)
        decode._heads = ProfilerAutograd(decode._heads,  # pylint: disable=protected-access
                                         device=getattr(args, 'device', 'cuda'),
                                         out_name=args.profile_decoder)
    return decode


def _meta(head):
    return getattr(head, 'meta', head)


def _stride(head, basenet_stride):
    """head_net.stride(basenet_stride) for a head network; a bare meta has none (then the
    FieldConfig default 8 stays)."""
    fn = getattr(head, 'stride', None)
    return fn(basenet_stride) if callable(fn) else None


def factory_decode(head_nets, *, basenet_stride, dense_coupling=0.0, dense_connections=False,
                   caf_seeds=False, multi_scale=False, multi_scale_hflip=True,
                   worker_pool=None):
    """Instantiate a decoder (factory.py:122-213).  head_nets are head networks with
    `.meta` and `.stride(basenet_stride)` or bare metas (duck-typed: a detection meta has
    `categories`, a keypoint meta `keypoints`, an association meta `skeleton`)."""
    assert not caf_seeds, 'not implemented'
    metas = [_meta(h) for h in head_nets]
    LOG.debug('head names = %s', tuple(getattr(m, 'name', '?') for m in metas))

    if hasattr(metas[0], 'categories') and not hasattr(metas[0], 'keypoints'):
        # DetectionMeta (factory.py:136-147): FieldConfig defaults (stride 8); the head's
        # stride only feeds the reference's visualizer
        return CifDet(FieldConfig(), metas[0].categories, worker_pool=worker_pool)

    if not (hasattr(metas[0], 'keypoints') and len(metas) > 1 and
            hasattr(metas[1], 'skeleton')):
        raise Exception('decoder unknown for head names: {}'.format(
            tuple(getattr(m, 'name', '?') for m in metas)))

    field_config = FieldConfig()
    if multi_scale:  # factory.py:153-168
        per = 2 if dense_connections else 3
        field_config.cif_indices = [v * per for v in range(5)]
        field_config.caf_indices = [v * per + 1 for v in range(5)]
        field_config.cif_min_scales = [0.0, 12.0, 16.0, 24.0, 40.0]
        field_config.caf_min_distances = [v * 3.0 for v in field_config.cif_min_scales]
        field_config.caf_max_distances = [160.0, 240.0, 320.0, 480.0, None]
    if multi_scale and multi_scale_hflip:  # factory.py:169-180
        per = 2 if dense_connections else 3
        field_config.cif_indices = [v * per for v in range(10)]
        field_config.caf_indices = [v * per + 1 for v in range(10)]
        field_config.cif_min_scales *= 2
        field_config.caf_min_distances *= 2
        field_config.caf_max_distances *= 2
    if multi_scale:  # single-scale keeps the FieldConfig default stride 8, as the reference
        strides = [_stride(h, basenet_stride) for h in head_nets]
        if any(strides[i] is None for i in field_config.cif_indices + field_config.caf_indices):
            raise ValueError('multi-scale decoding needs head networks with stride()')
        field_config.cif_strides = [strides[i] for i in field_config.cif_indices]
        field_config.caf_strides = [strides[i] for i in field_config.caf_indices]

    skeleton = metas[1].skeleton
    if dense_connections:  # factory.py:182-188 (extends the meta's list in place)
        field_config.confidence_scales = (
            [1.0 for _ in skeleton] + [dense_coupling for _ in metas[2].skeleton])
        skeleton += metas[2].skeleton
    return CifCaf(field_config, keypoints=metas[0].keypoints, skeleton=skeleton,
                  out_skeleton=metas[1].skeleton, worker_pool=worker_pool)
