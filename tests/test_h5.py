"""The reference's .h5 label files (picard/data_saver.py:24-109, data.py:1497-1525) written and read
through the HDF5 C library (deeppicarditeration_amd/h5.py); the HDF5 project's own h5dump, where
present, is the independent reader that pins the format."""
import os
import shutil
import subprocess

import numpy as np
import pytest
import torch

h5 = pytest.importorskip("deeppicarditeration_amd.h5")

try:
    h5._load()
except RuntimeError as e:  # pragma: no cover - image without libhdf5
    pytest.skip(str(e), allow_module_level=True)

H5DUMP = shutil.which("h5dump") or ("/opt/conda/bin/h5dump" if os.path.exists("/opt/conda/bin/h5dump") else None)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_saver_fills_rows_in_order_and_dataset_batches(tmp_path, dtype):
    rng = np.random.default_rng(0)
    tx, y = rng.standard_normal((10, 5)), rng.standard_normal((10, 7))
    p = h5.data_file(tmp_path, 4, 1)
    assert p == tmp_path / "data_iter_4" / "split_01.h5"
    s = h5.H5Saver(p, 10, [5, 7], ["tx", "u_ux"], dtype)
    s.save([torch.from_numpy(tx[:6]), torch.from_numpy(y[:6])], 6)
    with pytest.raises(ValueError, match="Not all data"):
        s.create_torch_dataset(4)
    s.save_np([tx[6:], y[6:]], 4)
    with pytest.raises(ValueError, match="overflow"):
        s.save_np([tx[:1], y[:1]], 1)
    ds = s.create_torch_dataset(4)
    assert len(ds) == 2  # the 2-row tail is dropped, as in the reference's H5Dataset
    b = list(ds)
    assert b[1][0].dtype == torch.from_numpy(np.zeros(1, dtype)).dtype
    np.testing.assert_array_equal(b[1][1].numpy(), y[4:8].astype(dtype))
    np.testing.assert_array_equal(h5.read_dataset(p, "tx"), tx.astype(dtype))


@pytest.mark.skipif(H5DUMP is None, reason="h5dump not available")
def test_files_read_back_by_h5dump(tmp_path):
    p = tmp_path / "split_00.h5"
    s = h5.H5Saver(p, 2, [3, 2], ["tx", "u_ux"], np.float32)
    s.save_np([np.array([[0.5, 1.0, -2.0], [3.25, 4.0, 5.5]]), np.array([[1.5, -0.25], [7.0, 8.0]])], 2)
    s.close()
    head = subprocess.run([H5DUMP, "-H", str(p)], capture_output=True, text=True, check=True).stdout
    assert 'DATASET "tx"' in head and 'DATASET "u_ux"' in head
    assert "H5T_IEEE_F32LE" in head and "( 2, 3 ) / ( 2, 3 )" in head and "( 2, 2 ) / ( 2, 2 )" in head
    body = subprocess.run([H5DUMP, "-d", "u_ux", "-y", "-w", "0", str(p)], capture_output=True, text=True,
                          check=True).stdout
    data = body[body.index("DATA {") + 6:body.index("}", body.index("DATA {"))]
    vals = [float(v) for v in data.replace(",", " ").split()]
    assert vals == [1.5, -0.25, 7.0, 8.0]
