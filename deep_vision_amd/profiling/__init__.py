"""profiling"""
