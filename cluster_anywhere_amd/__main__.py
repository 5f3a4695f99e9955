import sys

from .scripts.cli import main

sys.exit(main())
