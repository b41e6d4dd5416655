"""CPU restatement of the reference hot path -- test infrastructure only."""
