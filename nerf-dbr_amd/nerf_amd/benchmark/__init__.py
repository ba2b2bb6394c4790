"""Benchmark-renderer plugin interface, the MI355X plugin and the suite."""
