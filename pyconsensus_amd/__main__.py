"""``python -m pyconsensus_amd`` -- the reference CLI (pyconsensus/__init__.py:613-898) on the GPU."""
import sys

from .cli import main

sys.exit(main(sys.argv))
