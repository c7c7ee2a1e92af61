"""Convert the reference's ``<split>_IMAGES_<dataName>.hdf5`` to the ``.npy`` form that
imagecaptioningconvnext_amd.data.CaptionDataset memory-maps (run where h5py is installed).

    python tools/hdf5_to_npy.py DATA_FOLDER DATA_NAME [TRAIN VAL TEST]
"""
import os
import sys

import numpy as np


def main(folder, name, splits):
    import h5py
    for split in splits:
        src = os.path.join(folder, f"{split}_IMAGES_{name}.hdf5")
        with h5py.File(src, "r") as h:
            imgs = h["images"]
            out = np.lib.format.open_memmap(os.path.join(folder, f"{split}_IMAGES_{name}.npy"), mode="w+",
                                            dtype=np.uint8, shape=imgs.shape)
            for i in range(0, imgs.shape[0], 1024):
                out[i:i + 1024] = imgs[i:i + 1024]
            out.flush()
            print(split, imgs.shape, "captions_per_image", int(h.attrs["captions_per_image"]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:] or ["TRAIN", "VAL", "TEST"])
