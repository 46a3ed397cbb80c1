graph [
  node [
    id 0
    label "0"
    host_bandwidth_up "50 Mbit"
    host_bandwidth_down "50 Mbit"
  ]
  node [
    id 1
    label "1"
    host_bandwidth_up "70 Mbit"
    host_bandwidth_down "70 Mbit"
  ]
  node [
    id 2
    label "2"
    host_bandwidth_up "90 Mbit"
    host_bandwidth_down "90 Mbit"
  ]
  node [
    id 3
    label "3"
    host_bandwidth_up "110 Mbit"
    host_bandwidth_down "110 Mbit"
  ]
  node [
    id 4
    label "4"
    host_bandwidth_up "130 Mbit"
    host_bandwidth_down "130 Mbit"
  ]
  node [
    id 5
    label "5"
    host_bandwidth_up "100 Mbit"
    host_bandwidth_down "100 Mbit"
  ]
  edge [
    source 0
    target 1
    latency "112 ms"
    packet_loss 0.0
  ]
  edge [
    source 0
    target 2
    latency "94 ms"
    packet_loss 0.0
  ]
  edge [
    source 0
    target 3
    latency "76 ms"
    packet_loss 0.0
  ]
  edge [
    source 0
    target 4
    latency "58 ms"
    packet_loss 0.0
  ]
  edge [
    source 0
    target 0
    latency "90 ms"
    packet_loss 0.0
  ]
  edge [
    source 0
    target 5
    latency "1 ms"
    packet_loss 0.0
  ]
  edge [
    source 1
    target 2
    latency "94 ms"
    packet_loss 0.0
  ]
  edge [
    source 1
    target 3
    latency "76 ms"
    packet_loss 0.0
  ]
  edge [
    source 1
    target 4
    latency "58 ms"
    packet_loss 0.0
  ]
  edge [
    source 1
    target 1
    latency "72 ms"
    packet_loss 0.0
  ]
  edge [
    source 1
    target 5
    latency "1 ms"
    packet_loss 0.0
  ]
  edge [
    source 2
    target 3
    latency "76 ms"
    packet_loss 0.0
  ]
  edge [
    source 2
    target 4
    latency "58 ms"
    packet_loss 0.0
  ]
  edge [
    source 2
    target 2
    latency "54 ms"
    packet_loss 0.0
  ]
  edge [
    source 2
    target 5
    latency "1 ms"
    packet_loss 0.0
  ]
  edge [
    source 3
    target 4
    latency "58 ms"
    packet_loss 0.0
  ]
  edge [
    source 3
    target 3
    latency "40 ms"
    packet_loss 0.0
  ]
  edge [
    source 3
    target 5
    latency "1 ms"
    packet_loss 0.0
  ]
  edge [
    source 4
    target 4
    latency "40 ms"
    packet_loss 0.0
  ]
  edge [
    source 4
    target 5
    latency "1 ms"
    packet_loss 0.0
  ]
  edge [
    source 5
    target 5
    latency "1 ms"
    packet_loss 0.0
  ]
]
