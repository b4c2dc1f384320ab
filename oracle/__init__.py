"""Oracle package — TEST INFRASTRUCTURE ONLY (see oracle/oracle.py and DESIGN.md §Oracle)."""
