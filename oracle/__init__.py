"""TEST INFRASTRUCTURE ONLY: CPU restatement of the reference plugins (see oracle.h)."""
