"""Mirror: `src.database.graph` is `egraph_dropin.graph_service` (the same module object)."""
import sys

import egraph_dropin.graph_service as _impl

sys.modules[__name__] = _impl
