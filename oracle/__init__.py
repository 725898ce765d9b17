"""CPU restatement of the reference rules engine -- test infrastructure only."""
