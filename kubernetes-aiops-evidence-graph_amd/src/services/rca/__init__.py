"""RCA services: GPU rules engine and ranker."""
