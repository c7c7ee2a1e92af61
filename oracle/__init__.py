"""CPU ORACLE — test infrastructure, NOT part of the product.

A plain PyTorch-CPU (fp32/fp64) restatement of the reference's teacher-forced train step
(SURVEY.md §8a rows a1-a11), each function citing the reference file:line it follows.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this package, and only as the checker / CPU baseline.  The product path
(``imagecaptioningconvnext_amd``) never imports it and fails loudly without its HIP library.

Pinning:
  * decoders, loss, clip, Adam, DDP averaging: pinned against golden vectors produced by the
    real reference code in this container (tests/golden/, tools/gen_golden.py).
  * ConvNeXt encoder: the reference builds it from torchvision (absent here, un-vendored,
    version unpinned — the reference cites PyTorch 2.8 docs, i.e. torchvision ~0.23).  The
    restatement follows torchvision's published ConvNeXt definition and is pinned by its
    published known answers (parameter totals 28,589,128 / 88,591,464 / 197,767,336 and
    4.46 / 15.36 / 34.36 GFLOPS (=GMACs) at 224x224) — element-wise encoder parity is
    "parity unpinned" against torchvision itself.
"""
