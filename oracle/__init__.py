"""ORACLE -- test infrastructure only (see nerf_oracle.py).  Never imported by the product package."""
