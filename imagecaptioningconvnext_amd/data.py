"""COCO caption data in the reference's on-disk schema (dataLoader.py:15-56).

``CaptionDataset(dataFolder, dataName, split)`` reads the same files the reference's does:
``<split>_CAPTIONS_<dataName>.json`` and ``<split>_CAPLENS_<dataName>.json`` (captions already
encoded, ``captions_per_image`` per image) and the images ``<split>_IMAGES_<dataName>.hdf5``
('images' uint8 [N, 3, 256, 256], attribute 'captions_per_image').  h5py is not part of this
image, so the images may also be given as ``<split>_IMAGES_<dataName>.npy`` (same array; memory
mapped) -- ``tools/hdf5_to_npy.py`` converts where h5py exists.

Difference from the reference, by design: items keep the raw uint8 pixels (``raw=True``, the
default) and the GPU does ``/255`` + ImageNet normalisation inside the encoder's stem kernel
(``imgcap_convnext_stem_u8``), so a batch crosses PCIe as bytes (4x less than float32) and no
host thread runs the float transform.  ``raw=False`` (or a ``transform``) reproduces the
reference's float tensors exactly (``FloatTensor(img / 255.)`` then the transform).
"""
import json
import os

import numpy as np
import torch
from torch.utils.data import Dataset


def _open_images(folder, split, name):
    """(images array, captions_per_image or None, closer).  ``.npy`` is memory-mapped; HDF5 needs
    h5py.  Called lazily in each DataLoader worker (dataLoader.py:39-41): an HDF5 handle must not
    cross a fork."""
    base = os.path.join(folder, split + '_IMAGES_' + name)
    if os.path.exists(base + '.npy'):
        arr = np.load(base + '.npy', mmap_mode='r', allow_pickle=False)
        return arr, None, None
    try:
        import h5py
    except ImportError as e:  # the image format needs h5py; say how to get the .npy form instead
        raise FileNotFoundError(f"{base}.npy not found and h5py is not installed to read {base}.hdf5 "
                                "(convert once with tools/hdf5_to_npy.py where h5py exists)") from e
    h = h5py.File(base + '.hdf5', 'r')
    return h['images'], int(h.attrs['captions_per_image']), h.close


class CaptionDataset(Dataset):
    """dataLoader.py:15-56: TRAIN items are (img, caption, caplen); VAL / TEST items add the
    image's ``captions_per_image`` reference captions (for BLEU)."""

    def __init__(self, dataFolder, dataName, split, transform=None, raw=True, captions_per_image=None):
        self.split = split
        assert self.split in {'TRAIN', 'VAL', 'TEST'}
        self.dataFolder, self.dataName = dataFolder, dataName
        with open(os.path.join(dataFolder, self.split + '_CAPTIONS_' + dataName + '.json'), 'r') as j:
            self.captions = json.load(j)
        with open(os.path.join(dataFolder, self.split + '_CAPLENS_' + dataName + '.json'), 'r') as j:
            self.caplens = json.load(j)
        # open once for the image count / captions_per_image, then close: the handle is reopened
        # lazily per process in __getitem__ (dataLoader.py:39-41), never shared across a fork
        imgs, cpi, close = _open_images(dataFolder, split, dataName)
        n_imgs = len(imgs)
        if close is not None:
            close()
        del imgs
        self.imgs = None
        if captions_per_image is not None:
            cpi = captions_per_image
        if cpi is None:  # .npy images: the Karpathy files hold exactly cpi captions per image
            if len(self.captions) % n_imgs:
                raise ValueError("captions do not divide evenly over the images; pass captions_per_image")
            cpi = len(self.captions) // n_imgs
        self.cpi = cpi
        self.transform = transform
        self.raw = raw and transform is None
        self.dataset_size = len(self.captions)

    def __getitem__(self, i):
        if self.imgs is None:  # first item in this process (each DataLoader worker opens its own)
            self.imgs = _open_images(self.dataFolder, self.split, self.dataName)[0]
        u8 = np.asarray(self.imgs[i // self.cpi])
        if self.raw:
            img = torch.from_numpy(np.array(u8, dtype=np.uint8, copy=True))
        else:
            img = torch.FloatTensor(u8 / 255.)
            if self.transform is not None:
                img = self.transform(img)
        caption = torch.LongTensor(self.captions[i])
        caplen = torch.LongTensor([self.caplens[i]])
        if self.split == 'TRAIN':
            return img, caption, caplen
        start = (i // self.cpi) * self.cpi
        all_captions = torch.LongTensor(self.captions[start:start + self.cpi])
        return img, caption, caplen, all_captions

    def __len__(self):
        return self.dataset_size


def normalize(img_float):
    """torchvision Normalize(mean=[0.485, 0.456, 0.406], std=[0.229, 0.224, 0.225]) (train.py:152)
    on a [3, H, W] / [B, 3, H, W] float tensor (the ``raw=False`` transform)."""
    from .models.encoder import IMAGENET_MEAN, IMAGENET_STD
    m = torch.tensor(IMAGENET_MEAN, dtype=img_float.dtype).view(-1, 1, 1)
    s = torch.tensor(IMAGENET_STD, dtype=img_float.dtype).view(-1, 1, 1)
    return (img_float - m) / s
