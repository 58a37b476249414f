"""Decoder configuration and construction (decoder/factory.py:17-213).

cli()/configure() are the reference's: they write the same CLASS ATTRIBUTES, which the
device decoder reads at call time.  factory_decode() accepts the network's head metas
(duck-typed: .name/.keypoints/.skeleton for CIF/CAF heads) and builds a CifCaf.
"""
import logging

from .caf_scored import CafScored
from .cif_hr import CifHr
from .cif_seeds import CifSeeds
from .field_config import FieldConfig
from .generator.cifcaf import CifCaf
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
    nms.Keypoints.instance_threshold = args.instance_threshold
    nms.Keypoints.keypoint_threshold = args.keypoint_threshold


def factory_from_args(args, model):
    configure(args)
    return factory_decode(model.head_nets,
                          basenet_stride=model.base_net.stride,
                          dense_coupling=args.dense_coupling,
                          dense_connections=args.dense_connections,
                          caf_seeds=args.caf_seeds,
                          multi_scale=getattr(args, 'multi_scale', False),
                          multi_scale_hflip=getattr(args, 'multi_scale_hflip', True),
                          worker_pool=args.decoder_workers)


def _meta(head):
    return getattr(head, 'meta', head)


def factory_decode(head_nets, *, basenet_stride, dense_coupling=0.0, dense_connections=False,
                   caf_seeds=False, multi_scale=False, multi_scale_hflip=True,
                   worker_pool=None):
    """Instantiate a decoder (factory.py:122-213)."""
    assert not caf_seeds, 'not implemented'
    metas = [_meta(h) for h in head_nets]
    if hasattr(metas[0], 'categories') and not hasattr(metas[0], 'keypoints'):
        raise NotImplementedError('CifDet (detection heads) is not implemented yet')
    if multi_scale:
        raise NotImplementedError('multi-scale decoding is not implemented yet')
    if not (hasattr(metas[0], 'keypoints') and hasattr(metas[1], 'skeleton')):
        raise Exception('decoder unknown for head names: {}'.format(
            tuple(getattr(m, 'name', '?') for m in metas)))
    field_config = FieldConfig()
    stride = getattr(head_nets[0], 'stride', None)
    if callable(stride):
        field_config.cif_strides = [stride(basenet_stride)]
        field_config.caf_strides = [head_nets[1].stride(basenet_stride)]
    skeleton = metas[1].skeleton
    if dense_connections:
        # field_config.confidence_scales is built but never passed on (factory.py:184-211)
        skeleton += metas[2].skeleton
    return CifCaf(field_config, keypoints=metas[0].keypoints, skeleton=skeleton,
                  out_skeleton=metas[1].skeleton, worker_pool=worker_pool)
