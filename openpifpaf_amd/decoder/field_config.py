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

    def single_scale(self):
        """The device decoder covers the single-scale configuration (one CIF, one CAF
        head, no min-scale / distance masks).  Multi-scale fusion (factory.py:153-180) is
        the next row of SURVEY.md §8(f)."""
        if (len(self.cif_indices) != 1 or len(self.caf_indices) != 1
                or any(self.cif_min_scales) or any(self.caf_min_distances)
                or any(d is not None for d in self.caf_max_distances)):
            raise NotImplementedError('multi-scale field configurations are not implemented '
                                      'on the device decoder yet')
        if self.cif_strides[0] != self.caf_strides[0]:
            raise NotImplementedError('CIF and CAF strides must match')
        return self.cif_indices[0], self.caf_indices[0], int(self.cif_strides[0])
