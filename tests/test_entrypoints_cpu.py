"""Entry points keep the reference's CLI (train.py:59-65) and produce COCO-shaped batches."""
import train


def test_cli_flags_match_reference():
    a = train.parse(["--teacherForcing", "--lstmDecoder", "--startingLayer", "7", "--encoderLr", "3e-4"])
    assert a.teacherForcing and a.lstmDecoder and a.startingLayer == 7 and abs(a.encoderLr - 3e-4) < 1e-12
    assert a.checkpoint is None and a.embeddingName is None
    d = train.parse([])
    assert d.startingLayer == 5 and d.encoderLr == 1e-4 and not d.teacherForcing


def test_synthetic_batches_shape():
    imgs, caps, lens = next(train.synthetic_loader(1, 2, "cpu"))
    assert imgs.shape == (2, 3, 224, 224) and caps.shape == (2, 52) and lens.shape == (2, 1)
    assert (caps[:, 0] == train.VOCAB - 2).all() and (caps[:, -1] == train.VOCAB - 1).all()
    assert int(lens[0]) == 52


def test_testpy_cli_and_results_name_match_reference():
    """test.py:63-68 flags and the results CSV names of test.py:128-131."""
    import importlib.util
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("imgcap_testpy", os.path.join(root, "test.py"))
    testpy = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(testpy)
    a = testpy.parse(["--checkpoint", "x.pth.tar", "--lstmDecoder", "--startingLayer", "7"])
    assert a.checkpoint == "x.pth.tar" and a.lstmDecoder and a.startingLayer == 7 and a.embeddingName is None
    assert testpy.results_name(True, 7, None) == "test-lstmDecoder-TeacherForcing-Finetuning7.csv"
    assert testpy.results_name(False, None, None) == "test-TransformerDecoder-TeacherForcing-FinetuningNone-None.csv"
