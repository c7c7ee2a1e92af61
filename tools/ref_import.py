"""Import the read-only reference (/root/reference) in THIS container only.

Test-infrastructure helper for ``tools/gen_golden.py``: it never ships, never runs on the
GPU box, and nothing under ``imagecaptioningconvnext_amd/`` imports it.

The reference modules import packages that are absent here (torchvision, gensim, h5py,
nltk).  None of those names are used on the teacher-forced decoder / train-step path
(SURVEY.md §8c), so we register inert placeholder modules in ``sys.modules`` for them and
then import the reference files by path.  The reference's ``Encoder`` (which needs
torchvision's ConvNeXt and a weight download) cannot be constructed and is not imported.
"""
import importlib.util
import os
import sys
import types

REF = "/root/reference"


def _stub(name, **attrs):
    mod = types.ModuleType(name)
    mod.__dict__.update(attrs)
    sys.modules[name] = mod
    return mod


class _Placeholder:  # stands for names that exist only to be imported, never called
    def __init__(self, *a, **k):
        raise RuntimeError("placeholder for an absent third-party name")


def install_stubs():
    if "torchvision" not in sys.modules:
        tv = _stub("torchvision")
        tvm = _stub("torchvision.models", ConvNeXt_Base_Weights=_Placeholder,
                    convnext_base=_Placeholder)
        tvt = _stub("torchvision.transforms", Normalize=_Placeholder, Compose=_Placeholder)
        tv.models, tv.transforms = tvm, tvt
    if "gensim" not in sys.modules:
        g = _stub("gensim")
        g.downloader = _stub("gensim.downloader")
        g.models = _stub("gensim.models", KeyedVectors=_Placeholder)
    if "h5py" not in sys.modules:
        _stub("h5py", File=_Placeholder)
    if "nltk" not in sys.modules:
        n = _stub("nltk")
        n.translate = _stub("nltk.translate")
        n.translate.bleu_score = _stub("nltk.translate.bleu_score", corpus_bleu=_Placeholder)


def load(relpath, modname=None, argv=None):
    """Import ``/root/reference/<relpath>`` as a module (stubs installed first)."""
    install_stubs()
    if REF not in sys.path:
        sys.path.insert(0, REF)
    modname = modname or "ref_" + relpath.replace("/", "_").replace(".py", "")
    if modname in sys.modules:
        return sys.modules[modname]
    old_argv = sys.argv
    if argv is not None:
        sys.argv = argv
    try:
        spec = importlib.util.spec_from_file_location(modname, os.path.join(REF, relpath))
        mod = importlib.util.module_from_spec(spec)
        sys.modules[modname] = mod
        spec.loader.exec_module(mod)
    finally:
        sys.argv = old_argv
    return mod
