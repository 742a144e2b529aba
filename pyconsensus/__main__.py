"""``python -m pyconsensus`` -- the reference CLI (pyconsensus/__init__.py:613-898) on the GPU."""
import sys

from pyconsensus_amd.cli import main

sys.exit(main(sys.argv))
