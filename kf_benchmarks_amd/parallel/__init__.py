"""Data-parallel strategies and collectives over RCCL (xGMI)."""
