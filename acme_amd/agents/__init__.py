"""Agents (acme/agents): DQN on the MI355X learner core."""
