"""MI355X-native teacher-forced train step for ConvNeXt image captioning.

Drop-in for sa06840/ImageCaptioningConvNeXt's hot path: the ``models``
subpackage mirrors the reference's ``models/encoder.py``, ``models/decoder.py`` and
``models/transformerDecoder.py`` class surfaces and state-dict keys; the compute runs on
hand-written gfx950 HIP kernels in ``libimgcap_hip.so`` (C ABI: include/imgcap_abi.h).
"""
__version__ = "0.1.0"
