"""Mirror: `src.services.ingestion.normalizer` is `egraph_dropin.normalizer` (the same module object)."""
import sys

import egraph_dropin.normalizer as _impl

sys.modules[__name__] = _impl
