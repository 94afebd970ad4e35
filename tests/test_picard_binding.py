"""Host-side pieces of the reference binding (`deeppicarditeration_amd/picard_binding.py`) that need no
GPU: the generator class derived from the reference's `_OnlineDataGenerator`, and DATA.FLOAT's
dtype mapping (picard/config.py:131-144)."""
import pytest
import torch

from deeppicarditeration_amd.data import OnlineDataGenerator
from deeppicarditeration_amd.picard_binding import generator_class, label_dtype


class _ReferenceBase:  # stands for picard.data._OnlineDataGenerator
    def sample_with_gradients(self, n):
        raise AssertionError("the reference's method must not be reached")


def test_generator_class_is_an_instance_of_the_callers_base_and_dispatches_to_the_hip_path():
    cls = generator_class(_ReferenceBase)
    assert issubclass(cls, _ReferenceBase) and issubclass(cls, OnlineDataGenerator)
    # this package's methods come first in the MRO
    assert cls.sample_with_gradients is OnlineDataGenerator.sample_with_gradients
    assert cls.__name__ == OnlineDataGenerator.__name__
    assert generator_class(_ReferenceBase) is cls  # cached per (base, impl)


def test_generator_class_without_base_or_with_a_base_already_in_the_mro():
    assert generator_class(None) is OnlineDataGenerator
    assert generator_class(object) is OnlineDataGenerator


@pytest.mark.parametrize("name,dtype", [("double", torch.float64), ("float64", torch.float64), ("float", torch.float32),
                                        ("float32", torch.float32), ("Double", torch.float64),
                                        (torch.float64, torch.float64)])
def test_label_dtype_follows_data_float(name, dtype):
    assert label_dtype(name) == dtype


def test_label_dtype_defaults_to_torch_default_and_rejects_the_rest():
    assert label_dtype(None) == torch.get_default_dtype()
    with pytest.raises(ValueError):
        label_dtype("half")
