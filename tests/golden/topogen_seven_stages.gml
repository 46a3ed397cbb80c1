graph [
  node [
    id 0
    label "0"
    host_bandwidth_up "10 Mbit"
    host_bandwidth_down "10 Mbit"
  ]
  node [
    id 1
    label "1"
    host_bandwidth_up "151 Mbit"
    host_bandwidth_down "151 Mbit"
  ]
  node [
    id 2
    label "2"
    host_bandwidth_up "292 Mbit"
    host_bandwidth_down "292 Mbit"
  ]
  node [
    id 3
    label "3"
    host_bandwidth_up "433 Mbit"
    host_bandwidth_down "433 Mbit"
  ]
  node [
    id 4
    label "4"
    host_bandwidth_up "574 Mbit"
    host_bandwidth_down "574 Mbit"
  ]
  node [
    id 5
    label "5"
    host_bandwidth_up "715 Mbit"
    host_bandwidth_down "715 Mbit"
  ]
  node [
    id 6
    label "6"
    host_bandwidth_up "856 Mbit"
    host_bandwidth_down "856 Mbit"
  ]
  node [
    id 7
    label "7"
    host_bandwidth_up "100 Mbit"
    host_bandwidth_down "100 Mbit"
  ]
  edge [
    source 0
    target 1
    latency "257 ms"
    packet_loss 0.0
  ]
  edge [
    source 0
    target 2
    latency "215 ms"
    packet_loss 0.0
  ]
  edge [
    source 0
    target 3
    latency "173 ms"
    packet_loss 0.0
  ]
  edge [
    source 0
    target 4
    latency "131 ms"
    packet_loss 0.0
  ]
  edge [
    source 0
    target 5
    latency "89 ms"
    packet_loss 0.0
  ]
  edge [
    source 0
    target 6
    latency "47 ms"
    packet_loss 0.0
  ]
  edge [
    source 0
    target 0
    latency "294 ms"
    packet_loss 0.0
  ]
  edge [
    source 0
    target 7
    latency "1 ms"
    packet_loss 0.0
  ]
  edge [
    source 1
    target 2
    latency "215 ms"
    packet_loss 0.0
  ]
  edge [
    source 1
    target 3
    latency "173 ms"
    packet_loss 0.0
  ]
  edge [
    source 1
    target 4
    latency "131 ms"
    packet_loss 0.0
  ]
  edge [
    source 1
    target 5
    latency "89 ms"
    packet_loss 0.0
  ]
  edge [
    source 1
    target 6
    latency "47 ms"
    packet_loss 0.0
  ]
  edge [
    source 1
    target 1
    latency "252 ms"
    packet_loss 0.0
  ]
  edge [
    source 1
    target 7
    latency "1 ms"
    packet_loss 0.0
  ]
  edge [
    source 2
    target 3
    latency "173 ms"
    packet_loss 0.0
  ]
  edge [
    source 2
    target 4
    latency "131 ms"
    packet_loss 0.0
  ]
  edge [
    source 2
    target 5
    latency "89 ms"
    packet_loss 0.0
  ]
  edge [
    source 2
    target 6
    latency "47 ms"
    packet_loss 0.0
  ]
  edge [
    source 2
    target 2
    latency "210 ms"
    packet_loss 0.0
  ]
  edge [
    source 2
    target 7
    latency "1 ms"
    packet_loss 0.0
  ]
  edge [
    source 3
    target 4
    latency "131 ms"
    packet_loss 0.0
  ]
  edge [
    source 3
    target 5
    latency "89 ms"
    packet_loss 0.0
  ]
  edge [
    source 3
    target 6
    latency "47 ms"
    packet_loss 0.0
  ]
  edge [
    source 3
    target 3
    latency "168 ms"
    packet_loss 0.0
  ]
  edge [
    source 3
    target 7
    latency "1 ms"
    packet_loss 0.0
  ]
  edge [
    source 4
    target 5
    latency "89 ms"
    packet_loss 0.0
  ]
  edge [
    source 4
    target 6
    latency "47 ms"
    packet_loss 0.0
  ]
  edge [
    source 4
    target 4
    latency "126 ms"
    packet_loss 0.0
  ]
  edge [
    source 4
    target 7
    latency "1 ms"
    packet_loss 0.0
  ]
  edge [
    source 5
    target 6
    latency "47 ms"
    packet_loss 0.0
  ]
  edge [
    source 5
    target 5
    latency "84 ms"
    packet_loss 0.0
  ]
  edge [
    source 5
    target 7
    latency "1 ms"
    packet_loss 0.0
  ]
  edge [
    source 6
    target 6
    latency "42 ms"
    packet_loss 0.0
  ]
  edge [
    source 6
    target 7
    latency "1 ms"
    packet_loss 0.0
  ]
  edge [
    source 7
    target 7
    latency "1 ms"
    packet_loss 0.0
  ]
]
