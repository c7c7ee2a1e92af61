"""Static guard for the captured-schedule fault of round 3: the library issues
no memset / memcpy API calls on its launch paths, so a captured step holds kernel nodes only."""
import os
import re

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "imagecaptioningconvnext_amd", "csrc")


def test_library_launch_paths_issue_no_memset_or_memcpy_nodes():
    bad = []
    for name in sorted(os.listdir(CSRC)):
        if not name.endswith((".hip", ".cpp", ".h")):
            continue
        with open(os.path.join(CSRC, name)) as f:
            for i, line in enumerate(f, 1):
                code = line.split("//")[0]
                # hipMemcpyToSymbol of the diagnostic stamp pointer (host-side setup, never captured)
                if re.search(r"\bhipMemset\w*\s*\(|\bhipMemcpy(Async|2D\w*|Peer\w*)?\s*\(", code):
                    bad.append(f"{name}:{i}: {line.strip()}")
    assert not bad, bad
