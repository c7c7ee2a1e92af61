"""CaptionDataset in the reference's schema (dataLoader.py:15-56) on a synthetic dataset in
tmp: item layout, the i // captions_per_image image index, VAL/TEST reference captions, and the
reference's float transform (raw=False) vs the raw uint8 items the GPU normalises."""
import json
import os

import numpy as np
import torch


def _write(folder, split, name, n_img=3, cpi=5, L=12):
    rng = np.random.default_rng(0)
    imgs = rng.integers(0, 256, size=(n_img, 3, 16, 16), dtype=np.uint8)
    np.save(os.path.join(folder, f"{split}_IMAGES_{name}.npy"), imgs)
    caps = rng.integers(1, 40, size=(n_img * cpi, L)).tolist()
    lens = rng.integers(3, L, size=n_img * cpi).tolist()
    with open(os.path.join(folder, f"{split}_CAPTIONS_{name}.json"), "w") as f:
        json.dump(caps, f)
    with open(os.path.join(folder, f"{split}_CAPLENS_{name}.json"), "w") as f:
        json.dump(lens, f)
    return imgs, caps, lens


def test_caption_dataset_items(tmp_path):
    from imagecaptioningconvnext_amd.data import CaptionDataset, normalize
    imgs, caps, lens = _write(str(tmp_path), "TRAIN", "x")
    ds = CaptionDataset(str(tmp_path), "x", "TRAIN")
    assert len(ds) == 15 and ds.cpi == 5
    img, cap, cl = ds[7]
    assert img.dtype == torch.uint8 and torch.equal(img, torch.from_numpy(imgs[1]))
    assert cap.tolist() == caps[7] and cl.tolist() == [lens[7]]
    ref = CaptionDataset(str(tmp_path), "x", "TRAIN", transform=normalize)
    rimg, _, _ = ref[7]
    want = (torch.FloatTensor(imgs[1] / 255.) - torch.tensor([0.485, 0.456, 0.406]).view(3, 1, 1)) \
        / torch.tensor([0.229, 0.224, 0.225]).view(3, 1, 1)
    assert rimg.dtype == torch.float32 and torch.equal(rimg, want)


def test_caption_dataset_val_all_captions(tmp_path):
    from imagecaptioningconvnext_amd.data import CaptionDataset
    _, caps, _ = _write(str(tmp_path), "VAL", "x")
    ds = CaptionDataset(str(tmp_path), "x", "VAL")
    img, cap, cl, allc = ds[12]
    assert allc.tolist() == caps[10:15]
    loader = torch.utils.data.DataLoader(ds, batch_size=4, shuffle=False)
    b = next(iter(loader))
    assert b[0].shape == (4, 3, 16, 16) and b[0].dtype == torch.uint8 and b[3].shape == (4, 5, 12)


def test_caption_dataset_opens_images_lazily_per_worker(tmp_path):
    """dataLoader.py:39-41: no image handle is held after __init__, so forked DataLoader workers
    each open their own (an HDF5 handle must not cross a fork)."""
    import pickle
    from imagecaptioningconvnext_amd.data import CaptionDataset
    imgs, _, _ = _write(str(tmp_path), "TRAIN", "x")
    ds = CaptionDataset(str(tmp_path), "x", "TRAIN")
    assert ds.imgs is None
    clone = pickle.loads(pickle.dumps(ds))  # what a spawned worker receives
    assert torch.equal(clone[3][0], torch.from_numpy(imgs[0]))
    loader = torch.utils.data.DataLoader(ds, batch_size=5, shuffle=False, num_workers=2)
    got = torch.cat([b[0] for b in loader])
    assert torch.equal(got, torch.from_numpy(np.repeat(imgs, 5, axis=0)))
    assert ds.imgs is None  # the parent never opened it
