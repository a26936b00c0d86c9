"""Entry point: ``python -m parallel_heat_amd``."""
import sys

from .cli import main

sys.exit(main())
