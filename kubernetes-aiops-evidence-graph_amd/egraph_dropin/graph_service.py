"""Drop-in GraphService (reference src/database/neo4j.py:68-202) backed by the GPU snapshot.

Write path: create_entity / create_entities_batch / create_relation / create_relations_batch
keep the reference's MERGE semantics and return values (attempted counts, :112 / :166).
Read path: get_incident_graph(incident_id, depth=3) reproduces
`MATCH (i:Incident {id}) CALL apoc.path.subgraphAll(i, {maxLevel: depth})` (:170-202): the
vertex set within `depth` undirected hops (egr_plan_reach_hop on the device) and every edge
among those vertices (egr_plan_induced_edges).  As in the reference, the Incident vertex's id
property is the GraphEntity id ("incident:<uuid>", neo4j.py:101-102), so a bare UUID matches
nothing unless `resolve_bare_uuid=True`.

Root-cause ranking (build-defined): rank_root_causes runs
the frontier engine (egr_frontier_*) -- per incident, 3-hop typed propagation of the evidence
rows' signal strengths over the graph, ranked over the incident's 3-hop reach set.

The graph is process-wide, like the Neo4j database the reference talks to.  Writes go to the host
graph (MERGE); the next read brings the device snapshot up to date with ONE incremental update
(egr_snapshot_update: the appended vertices and edges merged into the CSR on the device) instead
of a rebuild and re-upload.

Concurrency: Temporal runs activities concurrently, and the ranking runs in a worker thread
(asyncio.to_thread) while writes arrive on the event loop.  Every access to the shared state --
the host graph (whose C++ vectors a write reallocates), the snapshot sync, the cached plans and
frontiers and their output buffers -- holds one process-wide lock, from the write or the
set_seeds through the read-back of the results.
"""
from __future__ import annotations

import asyncio
import threading
import time

import numpy as np
import torch

from egraph import ops
from egraph._lib import pyhost
from egraph.batcher import gc_paused
from egraph.device import to_device
from egraph.graph import EvidenceGraph
from egraph.seeds import seeds_for_batch
from egraph_dropin.models.evidence import GraphEntity, GraphRelation


class _StageClock:
    """Seconds per stage into `stages` (None: does nothing); a stage given a device ends with
    a device synchronise, so its device work is counted in it."""

    def __init__(self, stages: dict | None):
        self.stages = stages
        self.t = time.perf_counter() if stages is not None else 0.0

    def lap(self, name: str, dev=None) -> None:
        if self.stages is None:
            return
        if dev is not None:
            torch.cuda.synchronize(dev)
        t = time.perf_counter()
        self.stages[name] = self.stages.get(name, 0.0) + t - self.t
        self.t = t


class GraphService:
    """Service for Evidence Graph operations (process-wide store)."""

    _graph: EvidenceGraph | None = None
    _snapshot = None
    _plans: dict = {}
    _frontiers: dict = {}
    _lock = threading.RLock()
    device = None

    @classmethod
    def graph(cls) -> EvidenceGraph:
        if cls._graph is None:
            cls._graph = EvidenceGraph()
        return cls._graph

    @classmethod
    def reset(cls) -> None:
        with cls._lock:
            cls._graph, cls._snapshot, cls._plans, cls._frontiers = None, None, {}, {}

    @classmethod
    def _invalidate(cls) -> None:
        """After a write: the snapshot is synced lazily by the next read (_snap)."""

    @staticmethod
    async def create_entity(entity: GraphEntity) -> str:
        GraphService.create_entities_sync([entity])
        return entity.id

    @staticmethod
    async def create_entities_batch(entities: list[GraphEntity]) -> int:
        return GraphService.create_entities_sync(entities)

    @staticmethod
    async def create_relation(relation: GraphRelation) -> bool:
        with GraphService._lock:
            known = GraphService.graph().lookup([relation.source_id, relation.target_id])
            GraphService.create_relations_sync([relation])
        return bool((known >= 0).all())

    @staticmethod
    async def create_relations_batch(relations: list[GraphRelation]) -> int:
        return GraphService.create_relations_sync(relations)

    @classmethod
    def create_entities_sync(cls, entities) -> int:
        with cls._lock:
            n = cls.graph().create_entities_batch(entities)
            cls._invalidate()
        return n

    @classmethod
    def create_relations_sync(cls, relations) -> int:
        with cls._lock:
            n = cls.graph().create_relations_batch(relations)
            cls._invalidate()
        return n

    @classmethod
    def _plan(cls, n_cols: int):
        snap = cls._snap()          # syncs first: a write drops the plans
        if n_cols not in cls._plans:
            cls._plans[n_cols] = snap.plan(n_cols, max_seeds=0, k=1)
        return cls._plans[n_cols]

    @classmethod
    def _snap(cls):
        g = cls.graph()
        if cls._snapshot is None:
            cls._snapshot = g.snapshot(device=cls.device)
        elif cls._snapshot.sync(g) != (0, 0):
            cls._plans = {}        # plans are sized for one snapshot version
            cls._frontiers = {k: f for k, f in cls._frontiers.items()
                              if f.max_vertices >= cls._snapshot.n_vertices}
        return cls._snapshot

    @classmethod
    def _frontier(cls, n_cols: int, n_seeds: int, k: int):
        """A frontier for n_cols columns, reused while its seed capacity suffices."""
        snap = cls._snap()
        fr = cls._frontiers.get((n_cols, k))
        if fr is None or fr.max_seeds < n_seeds:
            fr = snap.frontier(n_cols, max_seeds=max(n_seeds, 1024), k=k, pool_entries=-1)
            cls._frontiers[(n_cols, k)] = fr
        return fr

    @staticmethod
    async def rank_root_causes(incident_ids: list[str], evidence_lists: list[list[dict]],
                               hops: int = 3, k: int = 10) -> list[list[dict]]:
        # the launch + completion wait run off the event loop (the worker is never blocked)
        return await asyncio.to_thread(GraphService.rank_root_causes_sync, incident_ids,
                                       evidence_lists, hops, k)

    @classmethod
    def rank_root_causes_sync(cls, incident_ids: list[str], evidence_lists: list[list[dict]],
                              hops: int = 3, k: int = 10, stages: dict | None = None) -> list[list[dict]]:
        """Per incident, the top-k graph entities by propagated evidence score, over the
        entities within `hops` undirected hops of the incident (Incident entities excluded):
        [{"id", "labels", "score", "rank"}], score descending, entity order on ties.
        Incidents are matched like get_incident_graph: by Incident id, or "incident:<id>".
        `stages` (a dict, diagnostics): filled with each host / device stage's seconds (the
        device is synchronised between stages, so the parts add up to the call)."""
        if len(incident_ids) != len(evidence_lists):
            raise ValueError("incident_ids and evidence_lists differ in length")
        if not incident_ids:
            return []
        with cls._lock:
            return cls._rank_locked(incident_ids, evidence_lists, hops, k, stages)

    @classmethod
    def _rank_locked(cls, incident_ids, evidence_lists, hops, k, stages=None):
        # (the cyclic GC deferred while the call builds its seed arrays and ~k entity dicts per
        # incident: collections triggered by those allocations traverse the whole heap -- the
        # graph's and the callers' evidence objects -- and find nothing to free)
        with gc_paused():
            return cls._rank_body(incident_ids, evidence_lists, hops, k, stages)

    @classmethod
    def _rank_body(cls, incident_ids, evidence_lists, hops, k, stages=None):
        g = cls.graph()
        if g.num_vertices == 0:
            return [[] for _ in incident_ids]
        clock = _StageClock(stages)
        ids = [str(i) for i in incident_ids]
        keys = g.lookup_labeled(ids, "Incident")
        miss = np.flatnonzero(keys < 0)
        if len(miss):                        # the collectors' prefixed form of a bare id
            keys[miss] = g.lookup_labeled([f"incident:{ids[j]}" for j in miss.tolist()], "Incident")
        keys = keys.tolist()
        clock.lap("incident_lookup")
        sv, sc, ss = seeds_for_batch(g, evidence_lists)
        clock.lap("seed_attach")
        fr = cls._frontier(len(keys), len(sv), k)
        dev = fr.dev
        clock.lap("snapshot_sync", dev)
        src = torch.tensor(keys, dtype=torch.int32, device=dev)   # -1 = EGR_NO_NODE: no column
        dsv, dsc, dss = to_device(sv, dev), to_device(sc, dev), to_device(ss, dev)
        clock.lap("upload", dev)
        labels = g.labels()
        inc = labels.index("Incident") if "Incident" in labels else -1
        # torch.ops.egraph.frontier_run: the registered custom op (seeds + run of the frontier)
        ids, scores = ops.frontier_run(fr, dsv, dsc, dss, src, hops, inc)
        clock.lap("device", dev)
        ids = ids.cpu().numpy().view("uint32")
        scores = scores.cpu().numpy()
        clock.lap("readback")
        fr.adapt()              # overflowing columns: the wide-table retry from the next call on
        clock.lap("adapt")
        # the ranked vertices' labels by numpy indexing (no per-vertex list of the whole graph),
        # then the entity dicts natively (csrc/pyhost.c entity_rows; the loop it replaces:
        # {"id": vid[v], "labels": [labels[label of v]], "score": score, "rank": r + 1} per
        # ranked vertex, each list up to its first EGR_NO_NODE)
        lab = np.zeros(ids.shape, np.uint8)
        ok = ids != 0xFFFFFFFF
        lab[ok] = g.vertex_labels()[ids[ok]]
        clock.lap("labels")
        out = pyhost.entity_rows(np.ascontiguousarray(ids), np.ascontiguousarray(scores, np.float32),
                                 lab, ids.shape[1] if ids.ndim == 2 else k, g._vertex_ids(), list(labels))
        clock.lap("entity_rows")
        return out

    @classmethod
    def save(cls, path) -> dict:
        """Checkpoint the process-wide graph (vertices, edges, properties, CSR) to a snapshot
        file (egraph/snapfile.py).  In the reference the worker (which writes the graph) and
        the ingestion service (which serves GET /graph) share one Neo4j server; here each
        process holds its graph, and a file written by one is what the other loads."""
        from egraph import snapfile
        with cls._lock:
            return snapfile.save(path, cls.graph())

    @classmethod
    def load(cls, path) -> None:
        """Replace the process-wide graph with a saved one (the device snapshot is rebuilt by
        the next read)."""
        from egraph import snapfile
        g = snapfile.load_graph(path)
        with cls._lock:
            cls._graph, cls._snapshot, cls._plans, cls._frontiers = g, None, {}, {}

    @staticmethod
    async def init_constraints() -> None:
        """Reference neo4j.py:299-321 creates uniqueness constraints on the id of Incident, Pod,
        Deployment, Service, Node and ChangeEvent plus two indexes.  Here MERGE already keys
        every vertex by (label, id) and the id index (egr_graph_find) is built with the graph,
        so this only creates the process-wide graph; called at ingestion startup
        (ingestion/main.py:55)."""
        GraphService.graph()

    @staticmethod
    async def cleanup_incident_graph(incident_id: str) -> int:
        """Reference neo4j.py:282-297: `MATCH (i:Incident {id}) CALL apoc.path.subgraphAll(i,
        {maxLevel: 10}) YIELD nodes DETACH DELETE nodes RETURN count(*)` -- every vertex within
        10 undirected hops of the incident is deleted with its relationships.  The query's
        count(*) counts result rows, not nodes: 1 when the incident exists, 0 when it does not;
        the same is returned here."""
        return GraphService.cleanup_incident_graph_sync(incident_id)

    @classmethod
    def cleanup_incident_graph_sync(cls, incident_id: str, max_level: int = 10) -> int:
        with cls._lock:
            g = cls.graph()
            v = g.vertex_of.get(("Incident", str(incident_id)))
            if v is None:
                return 0
            # deletion renumbers the vertices: the host graph is rebuilt without them and the
            # device snapshot, plans and frontiers are rebuilt by the next read
            cls._graph = g.subgraph(~g.within_hops(v, max_level))
            cls._snapshot, cls._plans, cls._frontiers = None, {}, {}
            return 1

    # ---- typed path queries (neo4j.py:205-279) ---------------------------------------------
    # Each Cypher MATCH step is one typed hop on the device snapshot (Snapshot.typed_neighbors,
    # egr_snapshot_typed_neighbors); properties come from the host graph, as the reference's
    # `dict(node)`.  Row semantics follow the Cypher text (oracle/graph_queries.py restates them
    # on an edge list): one row per matched path, OPTIONAL MATCH rows with None, collect(DISTINCT)
    # by first occurrence, the changed_at filter true only for timezone-aware datetimes (a Neo4j
    # DATETIME; strings and naive datetimes compare to null).  Neo4j leaves the order of
    # unordered rows unspecified; here it is match order: query vertices in vertex order,
    # neighbours in CSR order.
    # The (p)<-[:OWNS*]-(d) expansion runs until no open path is left, as Cypher's unbounded
    # variable-length match does: relationships are unique within a path, so it terminates.  A
    # relationship is identified by its (owner, owned) vertex pair: the reference writes every
    # relation with MERGE (source)-[r:TYPE]->(target) (neo4j.py:122, :152), so there is at most
    # one OWNS relationship per ordered pair and pair uniqueness is relationship uniqueness.

    @classmethod
    def _props(cls, g, labels, vlabel, v: int) -> dict:
        lab = labels[vlabel[v]]
        vid = g.vertex_id(int(v))
        return dict(g.node_props.get((lab, vid), {"id": vid}))

    @classmethod
    def _match_props(cls, g, label: str, **want) -> list[int]:
        """MATCH (n:label {k: v, ...}) on properties: the vertices in vertex order."""
        ids = [i for (lab, i), p in g.node_props.items()
               if lab == label and all(k in p and p[k] == x for k, x in want.items())]
        if not ids:
            return []
        vs = g.lookup_labeled(ids, label)
        return sorted(int(v) for v in vs if v >= 0)

    @staticmethod
    def _index(names: list[str], name: str) -> int:
        return names.index(name) if name in names else -1

    @staticmethod
    async def find_related_changes(incident_id: str, time_window_minutes: int = 30) -> list[dict]:
        # (in a worker thread: the body takes the service lock, which a ranking call holds for
        # its whole run, and waits on device copies -- the event loop stays free)
        return await asyncio.to_thread(GraphService.find_related_changes_sync, incident_id, time_window_minutes)

    @classmethod
    def find_related_changes_sync(cls, incident_id: str, time_window_minutes: int = 30,
                                  now=None) -> list[dict]:
        """MATCH (i:Incident {id})-[:AFFECTS]->(s), (s)<-[:APPLIES_TO]-(c:ChangeEvent) WHERE
        c.changed_at >= datetime() - duration({minutes}) RETURN c ORDER BY c.changed_at DESC
        (neo4j.py:205-229): the change events' property dicts."""
        import datetime as dt
        with cls._lock:
            g = cls.graph()
            if g.num_vertices == 0:
                return []
            incs = cls._match_props(g, "Incident", id=incident_id)
            labels, types = g.labels(), g.rel_types()
            ce = cls._index(labels, "ChangeEvent")
            if not incs or ce < 0:
                return []
            snap = cls._snap()
            targets = [s for row in snap.typed_neighbors(incs, cls._index(types, "AFFECTS"), snap.OUT)
                       for s in row.tolist()]
            changes = [c for row in snap.typed_neighbors(targets, cls._index(types, "APPLIES_TO"),
                                                         snap.IN, ce) for c in row.tolist()]
            vlabel = g.vertex_labels()
            cutoff = (now or dt.datetime.now(dt.timezone.utc)) - dt.timedelta(minutes=time_window_minutes)
            rows = []
            for c in changes:
                p = cls._props(g, labels, vlabel, c)
                t = p.get("changed_at")
                if isinstance(t, dt.datetime) and t.tzinfo is not None and t >= cutoff:
                    rows.append(p)
        rows.sort(key=lambda p: p["changed_at"], reverse=True)
        return rows

    @staticmethod
    async def find_affected_by_node(node_name: str) -> list[dict]:
        # (in a worker thread: the body takes the service lock, which a ranking call holds for
        # its whole run, and waits on device copies -- the event loop stays free)
        return await asyncio.to_thread(GraphService.find_affected_by_node_sync, node_name)

    @classmethod
    def find_affected_by_node_sync(cls, node_name: str) -> list[dict]:
        """MATCH (n:Node {name})<-[:SCHEDULED_ON]-(p:Pod), (p)<-[:OWNS*]-(d:Deployment)
        OPTIONAL MATCH (d)<-[:SELECTS]-(s:Service) RETURN p, d, s (neo4j.py:232-252):
        [{"pod", "deployment", "service" (None when no Service selects d)}], one per path."""
        with cls._lock:
            g = cls.graph()
            if g.num_vertices == 0:
                return []
            labels, types = g.labels(), g.rel_types()
            lp, ld, ls = (cls._index(labels, x) for x in ("Pod", "Deployment", "Service"))
            nodes = cls._match_props(g, "Node", name=node_name)
            if not nodes or lp < 0 or ld < 0:
                return []
            snap = cls._snap()
            t_owns = cls._index(types, "OWNS")
            vlabel = g.vertex_labels()
            pods = [p for row in snap.typed_neighbors(nodes, cls._index(types, "SCHEDULED_ON"), snap.IN, lp)
                    for p in row.tolist()]
            # OWNS* backwards from every pod, one level of every open path per launch; a path
            # is (its pod, its vertices' chain); relationships stay unique within a path
            paths = [(i, (p,)) for i, p in enumerate(pods)]
            found: list[list[tuple]] = [[] for _ in pods]   # per pod: (path vertices) ending at d
            while paths and t_owns >= 0:
                nb = snap.typed_neighbors([pv[-1] for _, pv in paths], t_owns, snap.IN)
                nxt = []
                for (i, pv), owners in zip(paths, nb):
                    used = set(zip(pv[1:], pv[:-1]))            # (owner, owned) edges on the path
                    for u in owners.tolist():
                        if (u, pv[-1]) in used:
                            continue
                        q = pv + (u,)
                        if vlabel[u] == ld:
                            found[i].append(q)
                        nxt.append((i, q))
                paths = nxt
            # per pod, the paths in depth-first order over CSR-ordered owners (lexicographic
            # order of the vertex chains: a path comes before its extensions)
            deps = [[q[-1] for q in sorted(f)] for f in found]
            flat_d = [d for ds in deps for d in ds]
            svcs = (snap.typed_neighbors(flat_d, cls._index(types, "SELECTS"), snap.IN, ls)
                    if flat_d and ls >= 0 else [np.empty(0, np.int64) for _ in flat_d])
            rows, j = [], 0
            for p, ds in zip(pods, deps):
                pp = cls._props(g, labels, vlabel, p)
                for d in ds:
                    dp = cls._props(g, labels, vlabel, d)
                    ss = svcs[j].tolist()
                    j += 1
                    for s in ss or [None]:
                        rows.append({"pod": dict(pp), "deployment": dict(dp),
                                     "service": cls._props(g, labels, vlabel, s) if s is not None else None})
        return rows

    @staticmethod
    async def get_service_dependencies(service_name: str, namespace: str) -> dict:
        # (in a worker thread: the body takes the service lock, which a ranking call holds for
        # its whole run, and waits on device copies -- the event loop stays free)
        return await asyncio.to_thread(GraphService.get_service_dependencies_sync, service_name, namespace)

    @classmethod
    def get_service_dependencies_sync(cls, service_name: str, namespace: str) -> dict:
        """MATCH (s:Service {name, namespace}) OPTIONAL MATCH (s)-[:CALLS]->(down:Service)
        OPTIONAL MATCH (up:Service)-[:CALLS]->(s) RETURN s, collect(DISTINCT down),
        collect(DISTINCT up) (neo4j.py:255-279), the first matching service's record."""
        none = {"service": None, "downstream": [], "upstream": []}
        with cls._lock:
            g = cls.graph()
            if g.num_vertices == 0:
                return none
            svc = cls._match_props(g, "Service", name=service_name, namespace=namespace)
            if not svc:
                return none
            labels, types = g.labels(), g.rel_types()
            ls, t_calls = cls._index(labels, "Service"), cls._index(types, "CALLS")
            snap = cls._snap()
            down = snap.typed_neighbors([svc[0]], t_calls, snap.OUT, ls)[0]
            up = snap.typed_neighbors([svc[0]], t_calls, snap.IN, ls)[0]
            vlabel = g.vertex_labels()

            def distinct(vs):
                return [cls._props(g, labels, vlabel, v) for v in dict.fromkeys(vs.tolist())]
            return {"service": cls._props(g, labels, vlabel, svc[0]),
                    "downstream": distinct(down), "upstream": distinct(up)}

    @staticmethod
    async def get_incident_graph(incident_id: str, depth: int = 3,
                                 resolve_bare_uuid: bool = False) -> dict:
        return (await asyncio.to_thread(GraphService.get_incident_graphs, [incident_id], depth,
                                        resolve_bare_uuid))[0]

    @classmethod
    def get_incident_graphs(cls, incident_ids: list[str], depth: int = 3,
                            resolve_bare_uuid: bool = False) -> list[dict]:
        """Batched get_incident_graph: one reach launch per hop for all incidents."""
        with cls._lock:
            return cls._graphs_locked(incident_ids, depth, resolve_bare_uuid)

    @classmethod
    def _graphs_locked(cls, incident_ids, depth, resolve_bare_uuid):
        g = cls.graph()
        empty = {"nodes": [], "relationships": []}
        if g.num_vertices == 0 or not incident_ids:
            return [dict(empty) for _ in incident_ids]
        ids = [str(i) for i in incident_ids]
        keys = g.lookup_labeled(ids, "Incident")
        miss = np.flatnonzero(keys < 0)
        if resolve_bare_uuid and len(miss):
            keys[miss] = g.lookup_labeled([f"incident:{ids[j]}" for j in miss.tolist()], "Incident")
        keys = keys.tolist()
        plan = cls._plan(len(keys))
        dev = plan.dev
        # -1 as int32 is EGR_NO_NODE as u32: an empty column
        src = torch.tensor([k if k >= 0 else -1 for k in keys], dtype=torch.int32, device=dev)
        plan.set_sources(src)
        for _ in range(depth):
            plan.reach_hop()
        bits = plan.read_reach().cpu().numpy().view("uint64")
        labels = g.labels()
        vlabel = g.vertex_labels()
        rtypes = g.rel_types()
        out = []
        for b, k in enumerate(keys):
            if k < 0:
                out.append(dict(empty))
                continue
            word = bits[b // 64]
            members = [int(v) for v in ((word >> (b % 64)) & 1).nonzero()[0]]
            nodes = []
            for v in members:
                lab = labels[vlabel[v]]
                vid = g.vertex_id(v)
                props = dict(g.node_props.get((lab, vid), {"id": vid}))
                nodes.append({"id": props.get("id"), "labels": [lab], "properties": props})
            rels = []
            for s, d, t in plan.induced_edges(b):
                sid, did = g.vertex_id(int(s)), g.vertex_id(int(d))
                rt = rtypes[int(t)]
                rels.append({"type": rt, "source": sid, "target": did,
                             "properties": dict(g.edge_props.get((sid, rt, did), {}))})
            out.append({"nodes": nodes, "relationships": rels})
        return out


class GraphConnection:
    """Stand-in for the reference's Neo4jConnection (neo4j.py:19-51), whose close() and
    verify_connectivity() the ingestion service calls at shutdown and in /health/ready
    (ingestion/main.py:60, :92).  There is no server: the graph lives in this process (host
    graph + device snapshot), and close() releases nothing, as closing a Neo4j driver leaves
    the database's contents in place."""

    @classmethod
    async def close(cls) -> None:
        return None

    @classmethod
    async def verify_connectivity(cls) -> bool:
        """True when the GPU the snapshot lives on is usable (False, as the reference returns
        on ServiceUnavailable, otherwise)."""
        try:
            return bool(torch.cuda.is_available())
        except Exception:  # noqa: BLE001
            return False


Neo4jConnection = GraphConnection     # the reference's name, for `from ... import Neo4jConnection`
