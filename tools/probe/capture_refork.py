"""Minimal forms of the capture topology that crashed hipStreamEndCapture in
tools/probe/dec_split.py (GPU box, diagnostics).  Inside one stream capture on M (torch's capture
stream), tiny kernels on side streams forked and joined with events (torch wait_stream):
  flat   : S forked from M, joined; X forked from M, joined (control)
  nested : S forked from M; X forked from S, joined to S; S joined to M
  nested_m : nested, plus a kernel on M between S's fork and join
  refork : nested_m, then X forked again from M and joined to M (dec_split's shape)
  fresh  : nested_m, then a fresh stream Y forked from M and joined to M
Prints "replay ok" or crashes in capture_end.  usage: python tools/probe/capture_refork.py VARIANT"""
import faulthandler
import sys

faulthandler.enable()
import torch  # noqa: E402

variant = sys.argv[1] if len(sys.argv) > 1 else "flat"
dev = torch.device("cuda:0")
a, b, c, d = (torch.zeros(1 << 16, device=dev) for _ in range(4))
S, X, Y = (torch.cuda.Stream(device=dev) for _ in range(3))


def body():
    M = torch.cuda.current_stream(dev)
    if variant == "flat":
        S.wait_stream(M)
        with torch.cuda.stream(S):
            a.add_(1.0)
        M.wait_stream(S)
        X.wait_stream(M)
        with torch.cuda.stream(X):
            b.add_(1.0)
        M.wait_stream(X)
        return
    S.wait_stream(M)
    with torch.cuda.stream(S):
        a.add_(1.0)
        X.wait_stream(S)
        with torch.cuda.stream(X):
            b.add_(1.0)
        S.wait_stream(X)
    if variant != "nested":
        c.add_(1.0)  # on M while S's branch is open
    if variant in ("refork", "fresh"):
        Z = X if variant == "refork" else Y
        Z.wait_stream(M)
        with torch.cuda.stream(Z):
            d.add_(1.0)
        M.wait_stream(Z)
    M.wait_stream(S)


body()
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    body()
print(f"{variant}: capture ended", flush=True)
g.replay()
torch.cuda.synchronize()
print(f"{variant}: replay ok", flush=True)
