"""Import the product package (directory `cuda.radixsort_amd/`, not a dotted package name)."""
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent.parent / "cuda.radixsort_amd"
if str(PKG) not in sys.path:
    sys.path.insert(0, str(PKG))

import radixsort as rs  # noqa: E402,F401


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
