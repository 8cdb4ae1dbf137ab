"""Bench / test harness pieces that are not part of the MI355X product package.

``orchestrator_contract`` drives an adapter the way the reference server's control plane
does (Morpheus_Client/orchestrator, SURVEY.md §2: reused as-is above the adapter), so the
shipped adapter and server can be measured and byte-pinned under that contract.
Deployments run the reference's own Orchestrator.
"""
