"""Reference-API mirror of the evidence-graph correlation path (drop-in for
ShreyashDarade/Kubernetes-AIOps-Evidence-Graph `src.*` on this path only)."""
