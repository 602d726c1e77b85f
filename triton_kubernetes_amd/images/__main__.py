import sys

from .packer import main

sys.exit(main())
