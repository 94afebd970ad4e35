"""A stand-in for the reference's `PicardDataModule` data path (picard/data.py:1411-1780), reduced
to the calls it makes on a label generator, so the drop-in can be driven exactly as the reference
drives it: `get_dataset_details` (:1620-1661) picks a `dataset*` method by the supervision flags,
`get_dataset_and_set_data_info` (:1714-1733) builds the dataset, `wrap_dataset` (:1746-1760)
caches it in memory for multi-epoch fits, `initialize_dataset` (:1510-1540) sizes it and attaches
the H5 saver, `train_dataloader` (:1762-1780) hands it to a DataLoader with `batch_size=None`.
Lightning, the memory probing of `NEW_SAMPLING` and DataLoader workers are left out (N_WORKERS = 0
in every shipped YAML).  Test infrastructure only."""
from collections import namedtuple

import numpy as np
from torch.utils.data import DataLoader

from deeppicarditeration_amd import dataset as D

Details = namedtuple("Details", ["dataset_fn", "data_dim", "data_name"])


class PicardDataModuleStandIn:
    def __init__(self, data_generator, nx, *, data_size, batch_size, n_batch_buffer, exact=False,
                 generate_gradients=True, generate_hessians=False, multi_epochs=False, shuffle=False, save_path=None,
                 float_type="single"):
        self.data_generator = data_generator
        self.nx = nx
        self.data_size = data_size
        self.batch_size = batch_size
        self.n_batch_buffer = n_batch_buffer
        self.exact = exact
        self.generate_gradients = generate_gradients
        self.generate_hessians = generate_hessians
        self.do_multi_epochs = multi_epochs
        self.shuffle = shuffle
        self.save_path = save_path
        self.float_type = float_type
        self.data_dim_input, self.data_name_input = 1 + nx, "tx"

    def get_dataset_details(self):
        flags = [k for k, on in (("exact", self.exact), ("gradient", self.generate_gradients),
                                 ("hessian", self.generate_hessians)) if on]
        g, nx = self.data_generator, self.nx
        table = {  # every entry is read eagerly, as in the reference
            "exact+gradient": Details(g.dataset_exact_with_gradients, 1 + nx, "u_ux"),
            "exact+gradient+hessian": Details(g.dataset_exact_with_gradients_and_hessians, 1 + nx + nx ** 2,
                                              "u_ux_uh"),
            "exact": Details(g.dataset_exact, 1, "u"),
            "gradient": Details(g.dataset_with_gradients, 1 + nx, "u_ux"),
            "gradient+hessian": Details(g.dataset_with_gradients_and_hessians, 1 + nx + nx ** 2, "u_ux_uh"),
            "": Details(g.dataset, 1, "u"),
        }
        return table["+".join(flags)]

    def get_dataset_and_set_data_info(self):
        dataset_fn, self.data_dim, self.data_name = self.get_dataset_details()
        self.active_data_size = self.data_size
        return dataset_fn(self.active_data_size, self.n_batch_buffer, self.batch_size)

    def wrap_dataset(self, dataset):
        if self.do_multi_epochs:
            assert self.data_generator.do_internal_batching
            assert isinstance(dataset, D.IterableDatasetWithInternalBatch)
            return D.CacheToMemoryWrapper(dataset, shuffle=self.shuffle)
        return dataset

    def initialize_dataset(self, dataset, worker_id=0, num_workers=1):
        n = self.active_data_size // num_workers
        h5_config = ()
        if self.save_path is not None:
            h5_config = (self.save_path, n, [self.data_dim_input, self.data_dim], [self.data_name_input, self.data_name],
                         np.float64 if self.float_type == "double" else np.float32)
        if isinstance(dataset, D.IterableDatasetWithInternalBatch):
            dataset.set_size(n)
            if h5_config:
                from deeppicarditeration_amd.h5 import H5Saver
                dataset.attach_saver(H5Saver(*h5_config))
        elif isinstance(dataset, D.CacheToMemoryWrapper):
            if h5_config:
                dataset.enable_save_to_file(h5_config)
            dataset.init(n, [1 + self.nx, self.data_dim], preload=False)
        else:
            raise NotImplementedError(type(dataset))

    def train_dataloader(self):
        dataset = self.wrap_dataset(self.get_dataset_and_set_data_info())
        self.initialize_dataset(dataset)
        return DataLoader(dataset, batch_size=None if self.data_generator.do_internal_batching else self.batch_size,
                          num_workers=0)
