"""Reference-compatible model classes (models/encoder.py, models/decoder.py,
models/transformerDecoder.py of sa06840/ImageCaptioningConvNeXt)."""
