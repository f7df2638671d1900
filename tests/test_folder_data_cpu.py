"""Real-image folder path (MX_DATA=folder:<root>) with the reference's transforms."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _make_tree(root, classes=3, per=4, size=(48, 40)):
    from PIL import Image
    rng = np.random.default_rng(0)
    for split in ("train", "val"):
        for c in range(classes):
            d = os.path.join(root, split, f"n{c:08d}")
            os.makedirs(d, exist_ok=True)
            for i in range(per):
                a = (rng.random((size[1], size[0], 3)) * 255).astype(np.uint8)
                Image.fromarray(a).save(os.path.join(d, f"img{i}.png"))


def test_imagefolder_and_transforms(tmp_path):
    from pytorch_distributed_amd.data.folder import ImageFolder, train_transform, val_transform
    _make_tree(str(tmp_path))
    ds = ImageFolder(str(tmp_path), "train", train_transform(32))
    assert len(ds) == 12 and ds.classes[0] == "n00000000"
    x, y = ds[5]
    assert x.shape == (3, 32, 32) and x.dtype == torch.float32 and y == 1
    vs = ImageFolder(str(tmp_path), "val", val_transform(32, 36))
    xv, _ = vs[0]
    assert xv.shape == (3, 32, 32)
    # val transform is deterministic
    assert torch.equal(vs[0][0], xv)
    ld = ds.loader(5, num_workers=0)
    batches = list(ld.iter_from(1))
    assert len(ld) == 3 and len(batches) == 2 and batches[0][0] == 1
    assert batches[-1][1][0].shape == (2, 3, 32, 32)


def test_cli_with_folder_data(tmp_path):
    _make_tree(str(tmp_path / "data"))
    env = dict(os.environ)
    env.update({"MX_ARCH": "resnet18", "MX_EPOCHS": "1", "MX_BATCH": "4", "MX_IMAGE_SIZE": "32",
                "MX_DEVICE": "cpu", "MX_DATA": f"folder:{tmp_path / 'data'}", "MX_WORKERS": "0",
                "PYTHONPATH": ROOT, "OMP_NUM_THREADS": "2"})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "resnet_single_gpu.py")], cwd=tmp_path,
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "Epoch: 0, Loss: " in r.stdout and "cost time per epoch" in r.stdout
