"""FieldConfig: which fields of the network output the decoder reads (field_config.py:5-25)."""
import dataclasses
from typing import List


@dataclasses.dataclass
class FieldConfig:
    cif_indices: List[int] = dataclasses.field(default_factory=lambda: [0])
    caf_indices: List[int] = dataclasses.field(default_factory=lambda: [1])
    cif_strides: List[int] = dataclasses.field(default_factory=lambda: [8])
    caf_strides: List[int] = dataclasses.field(default_factory=lambda: [8])
    cif_min_scales: List[float] = dataclasses.field(default_factory=lambda: [0.0])
    caf_min_distances: List[float] = dataclasses.field(default_factory=lambda: [0.0])
    caf_max_distances: List[float] = dataclasses.field(default_factory=lambda: [None])
    seed_mask: List[int] = None
    confidence_scales: List[float] = None
    cif_visualizers: list = None
    caf_visualizers: list = None

    def verify(self):
        assert len(self.cif_strides) == len(self.cif_indices)
        assert len(self.cif_strides) == len(self.cif_min_scales)
        assert len(self.caf_strides) == len(self.caf_indices)
        assert len(self.caf_strides) == len(self.caf_min_distances)
        assert len(self.caf_strides) == len(self.caf_max_distances)

    def is_single_scale(self):
        """One CIF and one CAF head at one stride without min-scale / distance masks: the
        pp_decode_stages path.  Everything else runs pp_decode_multi."""
        return (len(self.cif_indices) == 1 and len(self.caf_indices) == 1
                and not any(self.cif_min_scales) and not any(self.caf_min_distances)
                and all(d is None or not d for d in self.caf_max_distances)
                and self.cif_strides[0] == self.caf_strides[0])

    def single_scale(self):
        """(cif index, caf index, stride) of a single-scale configuration."""
        if not self.is_single_scale():
            raise NotImplementedError('not a single-scale field configuration')
        return self.cif_indices[0], self.caf_indices[0], int(self.cif_strides[0])
