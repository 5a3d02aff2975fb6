"""casadi stub: imported by multiagent/safety_filter.py:10 but never used."""
