import sys

from .serve import main

sys.exit(main())
