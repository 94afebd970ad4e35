"""The reference's on-disk label format: `data_iter_{i}/split_{w:02d}.h5`, one
HDF5 file per data worker with two 2-D datasets in the root group, `tx` (N, 1+nx) and the labels
(`u_ux` (N, 1+nx), or `u_ux_uh` (N, 1+nx+nx^2) with Hessian labels) — `picard/data_saver.py:24-56`
(`H5Saver`: create the datasets at full size, fill rows in order), `:86-109` (`H5Dataset`: batches
of `batch_size` rows), `picard/data.py:1497-1525, 1629-1660` (paths, names, dims).

h5py is not installed in this image, so this binds the HDF5 C library directly (ctypes; found via
$DPI_LIBHDF5, then the usual library names).  Files are plain HDF5 datasets of the requested fp
type, readable by h5py / h5dump exactly like the reference's (`tests/test_h5.py` checks them with
the HDF5 project's own `h5dump` where it is present).  Host-side only: the labels are copied off
the device once per `save`.
"""
import ctypes
import ctypes.util
import glob
import os
import pathlib

import numpy as np
import torch

_hid = ctypes.c_int64  # hid_t (HDF5 >= 1.10)
_hsize = ctypes.c_ulonglong
_H5F_ACC_RDONLY, _H5F_ACC_TRUNC = 0x0000, 0x0002
_H5P_DEFAULT = _H5S_ALL = 0
_H5S_SELECT_SET = 0
_lib = None


def _load():
    global _lib
    if _lib is not None:
        return _lib
    cands = [os.environ.get("DPI_LIBHDF5")] if os.environ.get("DPI_LIBHDF5") else []
    found = ctypes.util.find_library("hdf5")
    if found:
        cands.append(found)
    for d in ("/opt/conda/lib", "/usr/lib/x86_64-linux-gnu/hdf5/serial", "/usr/lib/x86_64-linux-gnu", "/usr/lib"):
        cands += sorted(glob.glob(os.path.join(d, "libhdf5.so*")))
    err = None
    for c in cands:
        try:
            h = ctypes.CDLL(c)
            break
        except OSError as e:  # try the next candidate
            err = e
    else:
        raise RuntimeError(f"the HDF5 C library is required for the .h5 label files (set DPI_LIBHDF5): {err}")
    if h.H5open() < 0:
        raise RuntimeError("H5open failed")
    sig = {
        "H5Fcreate": (_hid, [ctypes.c_char_p, ctypes.c_uint, _hid, _hid]),
        "H5Fopen": (_hid, [ctypes.c_char_p, ctypes.c_uint, _hid]),
        "H5Fclose": (ctypes.c_int, [_hid]),
        "H5Screate_simple": (_hid, [ctypes.c_int, ctypes.POINTER(_hsize), ctypes.POINTER(_hsize)]),
        "H5Sclose": (ctypes.c_int, [_hid]),
        "H5Sselect_hyperslab": (ctypes.c_int, [_hid, ctypes.c_int, ctypes.POINTER(_hsize), ctypes.POINTER(_hsize),
                                               ctypes.POINTER(_hsize), ctypes.POINTER(_hsize)]),
        "H5Sget_simple_extent_ndims": (ctypes.c_int, [_hid]),
        "H5Sget_simple_extent_dims": (ctypes.c_int, [_hid, ctypes.POINTER(_hsize), ctypes.POINTER(_hsize)]),
        "H5Dcreate2": (_hid, [_hid, ctypes.c_char_p, _hid, _hid, _hid, _hid, _hid]),
        "H5Dopen2": (_hid, [_hid, ctypes.c_char_p, _hid]),
        "H5Dclose": (ctypes.c_int, [_hid]),
        "H5Dget_space": (_hid, [_hid]),
        "H5Dget_type": (_hid, [_hid]),
        "H5Dwrite": (ctypes.c_int, [_hid, _hid, _hid, _hid, _hid, ctypes.c_void_p]),
        "H5Dread": (ctypes.c_int, [_hid, _hid, _hid, _hid, _hid, ctypes.c_void_p]),
        "H5Tget_size": (ctypes.c_size_t, [_hid]),
        "H5Tclose": (ctypes.c_int, [_hid]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(h, name)
        fn.restype, fn.argtypes = res, args
    _lib = h
    return h


def _native(dtype):
    h = _load()
    name = {np.dtype(np.float32): "H5T_NATIVE_FLOAT_g", np.dtype(np.float64): "H5T_NATIVE_DOUBLE_g"}.get(np.dtype(dtype))
    if name is None:
        raise TypeError(f"label files hold float32 or float64 (got {dtype})")
    return _hid.in_dll(h, name).value


def _ok(rc, what):
    if rc < 0:
        raise RuntimeError(f"HDF5: {what} failed")
    return rc


def _dims(*v):
    return (_hsize * len(v))(*v)


def data_file(exp_dir, i, worker=0):
    """picard/data.py:1497-1498, 1515: <exp_dir>/data_iter_{i}/split_{worker:02d}.h5."""
    d = pathlib.Path(exp_dir) / f"data_iter_{i}"
    d.mkdir(parents=True, exist_ok=True)
    return d / f"split_{worker:02d}.h5"


class H5Saver:
    """picard/data_saver.py:24-56: datasets `labels[k]` of shape (n_total, n_dims[k]) created up front,
    rows filled in order by save()."""

    def __init__(self, save_file_path, n_total, n_dims, labels, dtype):
        h = _load()
        self.save_file_path = str(save_file_path)
        self.labels = list(labels)
        self.dtype = np.dtype(dtype)
        self.n_total, self.n_dims = int(n_total), [int(d) for d in n_dims]
        self.f = _ok(h.H5Fcreate(self.save_file_path.encode(), _H5F_ACC_TRUNC, _H5P_DEFAULT, _H5P_DEFAULT), "H5Fcreate")
        self.dataset = []
        for d, name in zip(self.n_dims, self.labels):
            sp = _ok(h.H5Screate_simple(2, _dims(self.n_total, d), None), "H5Screate_simple")
            self.dataset.append(_ok(h.H5Dcreate2(self.f, name.encode(), _native(self.dtype), sp, _H5P_DEFAULT,
                                                 _H5P_DEFAULT, _H5P_DEFAULT), f"H5Dcreate2({name})"))
            h.H5Sclose(sp)
        self.position = 0

    def save(self, data, length: int):
        self.save_np([d.detach().cpu().numpy() if isinstance(d, torch.Tensor) else d for d in data], length)

    def save_np(self, data, length: int):
        h = _load()
        if self.position + length > self.n_total:
            raise ValueError(f"saver holds {self.n_total} rows; {self.position} + {length} would overflow it")
        for ds, d, w in zip(self.dataset, data, self.n_dims):
            a = np.ascontiguousarray(np.asarray(d)[:length], dtype=self.dtype)
            if a.shape != (length, w):
                raise ValueError(f"expected ({length}, {w}) rows, got {a.shape}")
            fsp = _ok(h.H5Dget_space(ds), "H5Dget_space")
            _ok(h.H5Sselect_hyperslab(fsp, _H5S_SELECT_SET, _dims(self.position, 0), None, _dims(length, w), None),
                "H5Sselect_hyperslab")
            msp = _ok(h.H5Screate_simple(2, _dims(length, w), None), "H5Screate_simple")
            _ok(h.H5Dwrite(ds, _native(self.dtype), msp, fsp, _H5P_DEFAULT, a.ctypes.data), "H5Dwrite")
            h.H5Sclose(msp)
            h.H5Sclose(fsp)
        self.position += length

    def close(self):
        if getattr(self, "f", None) is not None:
            h = _load()
            for ds in self.dataset:
                h.H5Dclose(ds)
            _ok(h.H5Fclose(self.f), "H5Fclose")
            self.f = None

    def create_torch_dataset(self, batch_size):
        if self.position < self.n_total:
            raise ValueError("Not all data are filled.")
        self.close()
        return H5Dataset(self.save_file_path, batch_size, self.labels)

    def __del__(self):
        self.close()


def read_dataset(path, name):
    """The whole dataset `name` of an .h5 label file as a numpy array of its stored fp type."""
    h = _load()
    f = _ok(h.H5Fopen(str(path).encode(), _H5F_ACC_RDONLY, _H5P_DEFAULT), "H5Fopen")
    try:
        ds = _ok(h.H5Dopen2(f, name.encode(), _H5P_DEFAULT), f"H5Dopen2({name})")
        sp = h.H5Dget_space(ds)
        nd = h.H5Sget_simple_extent_ndims(sp)
        dims = (_hsize * nd)()
        h.H5Sget_simple_extent_dims(sp, dims, None)
        t = h.H5Dget_type(ds)
        dtype = np.float64 if h.H5Tget_size(t) == 8 else np.float32
        h.H5Tclose(t)
        out = np.empty(tuple(dims), dtype=dtype)
        _ok(h.H5Dread(ds, _native(dtype), _H5S_ALL, _H5S_ALL, _H5P_DEFAULT, out.ctypes.data), "H5Dread")
        h.H5Sclose(sp)
        h.H5Dclose(ds)
        return out
    finally:
        h.H5Fclose(f)


class H5Dataset(torch.utils.data.IterableDataset):
    """picard/data_saver.py:86-109: yields [tx, labels] batches of batch_size rows (the tail that
    does not fill a batch is dropped, as there)."""

    def __init__(self, save_file_path, batch_size, labels):
        self.save_file_path, self.batch_size, self.labels = str(save_file_path), int(batch_size), list(labels)
        self.dataset = [read_dataset(self.save_file_path, la) for la in self.labels]
        self.len = len(self.dataset[0]) // self.batch_size

    def __iter__(self):
        for i in range(self.len):
            yield [torch.from_numpy(d[i * self.batch_size:(i + 1) * self.batch_size]) for d in self.dataset]

    def __len__(self):
        return self.len
