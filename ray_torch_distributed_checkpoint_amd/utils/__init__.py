"""Profiling (AMD SMI sampler + roctx phase ranges) and whole-step hipGraph capture helpers."""
