"""Mirror: `src.services.ingestion.deduplicator` is `egraph_dropin.deduplicator` (the same module object)."""
import sys

import egraph_dropin.deduplicator as _impl

sys.modules[__name__] = _impl
