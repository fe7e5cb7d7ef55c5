import sys

from .app.sphexa import main

sys.exit(main())
