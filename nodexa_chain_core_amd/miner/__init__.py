"""miner"""
