from ome_amd.router.server import main

raise SystemExit(main())
