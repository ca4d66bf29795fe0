"""Compatibility entry point with the reference's worker filename
(``llmctl/runtime/train_script.py``); the implementation is :mod:`llmctl.runtime.worker`."""

import sys

from llmctl.runtime.worker import main

if __name__ == "__main__":
    sys.exit(main())
