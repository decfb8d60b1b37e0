"""Research-question analyses declared by the reference's experiment spec (RQ2 resource efficiency and cost,
RQ3 operational complexity; /root/reference/experiment.yaml:38-60)."""
from .rq import complexity_report, cost_per_1000_requests, enrich_sweep_rows

__all__ = ["complexity_report", "cost_per_1000_requests", "enrich_sweep_rows"]
