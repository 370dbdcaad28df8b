graph [
  directed 0
  node [
    id 0
    ip_address "11.0.0.1"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 1
    ip_address "11.0.0.2"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 2
    ip_address "11.0.0.3"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 3
    ip_address "11.0.0.4"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 4
    ip_address "11.0.0.5"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 5
    ip_address "11.0.0.6"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 6
    ip_address "11.0.0.7"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 7
    ip_address "11.0.0.8"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 8
    ip_address "11.0.0.9"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 9
    ip_address "11.0.0.10"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 10
    ip_address "11.0.0.11"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 11
    ip_address "11.0.0.12"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 12
    ip_address "11.0.0.13"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 13
    ip_address "11.0.0.14"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 14
    ip_address "11.0.0.15"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 15
    ip_address "11.0.0.16"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 16
    ip_address "11.0.0.17"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 17
    ip_address "11.0.0.18"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 18
    ip_address "11.0.0.19"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 19
    ip_address "11.0.0.20"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 20
    ip_address "11.0.0.21"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 21
    ip_address "11.0.0.22"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 22
    ip_address "11.0.0.23"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 23
    ip_address "11.0.0.24"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 24
    ip_address "11.0.0.25"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 25
    ip_address "11.0.0.26"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 26
    ip_address "11.0.0.27"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 27
    ip_address "11.0.0.28"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 28
    ip_address "11.0.0.29"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 29
    ip_address "11.0.0.30"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 30
    ip_address "11.0.0.31"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 31
    ip_address "11.0.0.32"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 32
    ip_address "11.0.0.33"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 33
    ip_address "11.0.0.34"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 34
    ip_address "11.0.0.35"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 35
    ip_address "11.0.0.36"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 36
    ip_address "11.0.0.37"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 37
    ip_address "11.0.0.38"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 38
    ip_address "11.0.0.39"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 39
    ip_address "11.0.0.40"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 40
    ip_address "11.0.0.41"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 41
    ip_address "11.0.0.42"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 42
    ip_address "11.0.0.43"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 43
    ip_address "11.0.0.44"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 44
    ip_address "11.0.0.45"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 45
    ip_address "11.0.0.46"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 46
    ip_address "11.0.0.47"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 47
    ip_address "11.0.0.48"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 48
    ip_address "11.0.0.49"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  node [
    id 49
    ip_address "11.0.0.50"
    country_code "US"
    bandwidth_down "1 Gbit"
    bandwidth_up "1 Gbit"
  ]
  edge [
    source 0
    target 0
    latency "2 ms"
    packet_loss 0.0195
  ]
  edge [
    source 0
    target 1
    latency "156 ms"
    packet_loss 0.0136
  ]
  edge [
    source 0
    target 2
    latency "56 ms"
    packet_loss 0.0462
  ]
  edge [
    source 0
    target 3
    latency "179 ms"
    packet_loss 0.0186
  ]
  edge [
    source 0
    target 4
    latency "261 ms"
    packet_loss 0.0093
  ]
  edge [
    source 0
    target 5
    latency "77 ms"
    packet_loss 0.0366
  ]
  edge [
    source 0
    target 6
    latency "136 ms"
    packet_loss 0.0211
  ]
  edge [
    source 0
    target 7
    latency "223 ms"
    packet_loss 0.01
  ]
  edge [
    source 0
    target 8
    latency "110 ms"
    packet_loss 0.0263
  ]
  edge [
    source 0
    target 9
    latency "230 ms"
    packet_loss 0.0371
  ]
  edge [
    source 0
    target 10
    latency "25 ms"
    packet_loss 0.0129
  ]
  edge [
    source 0
    target 11
    latency "10 ms"
    packet_loss 0.0138
  ]
  edge [
    source 0
    target 12
    latency "285 ms"
    packet_loss 0.0097
  ]
  edge [
    source 0
    target 13
    latency "40 ms"
    packet_loss 0.0197
  ]
  edge [
    source 0
    target 14
    latency "261 ms"
    packet_loss 0.044
  ]
  edge [
    source 0
    target 15
    latency "80 ms"
    packet_loss 0.0237
  ]
  edge [
    source 0
    target 16
    latency "258 ms"
    packet_loss 0.0273
  ]
  edge [
    source 0
    target 17
    latency "53 ms"
    packet_loss 0.017
  ]
  edge [
    source 0
    target 18
    latency "140 ms"
    packet_loss 0.029
  ]
  edge [
    source 0
    target 19
    latency "32 ms"
    packet_loss 0.0498
  ]
  edge [
    source 0
    target 20
    latency "219 ms"
    packet_loss 0.018
  ]
  edge [
    source 0
    target 21
    latency "110 ms"
    packet_loss 0.0191
  ]
  edge [
    source 0
    target 22
    latency "41 ms"
    packet_loss 0.0139
  ]
  edge [
    source 0
    target 23
    latency "117 ms"
    packet_loss 0.0418
  ]
  edge [
    source 0
    target 24
    latency "217 ms"
    packet_loss 0.0017
  ]
  edge [
    source 0
    target 25
    latency "293 ms"
    packet_loss 0.0274
  ]
  edge [
    source 0
    target 26
    latency "144 ms"
    packet_loss 0.0038
  ]
  edge [
    source 0
    target 27
    latency "78 ms"
    packet_loss 0.0054
  ]
  edge [
    source 0
    target 28
    latency "244 ms"
    packet_loss 0.0432
  ]
  edge [
    source 0
    target 29
    latency "23 ms"
    packet_loss 0.0252
  ]
  edge [
    source 0
    target 30
    latency "11 ms"
    packet_loss 0.0466
  ]
  edge [
    source 0
    target 31
    latency "25 ms"
    packet_loss 0.0009
  ]
  edge [
    source 0
    target 32
    latency "196 ms"
    packet_loss 0.0165
  ]
  edge [
    source 0
    target 33
    latency "11 ms"
    packet_loss 0.0467
  ]
  edge [
    source 0
    target 34
    latency "92 ms"
    packet_loss 0.0399
  ]
  edge [
    source 0
    target 35
    latency "133 ms"
    packet_loss 0.0488
  ]
  edge [
    source 0
    target 36
    latency "31 ms"
    packet_loss 0.0384
  ]
  edge [
    source 0
    target 37
    latency "69 ms"
    packet_loss 0.0473
  ]
  edge [
    source 0
    target 38
    latency "124 ms"
    packet_loss 0.019
  ]
  edge [
    source 0
    target 39
    latency "236 ms"
    packet_loss 0.0302
  ]
  edge [
    source 0
    target 40
    latency "295 ms"
    packet_loss 0.0396
  ]
  edge [
    source 0
    target 41
    latency "183 ms"
    packet_loss 0.0459
  ]
  edge [
    source 0
    target 42
    latency "120 ms"
    packet_loss 0.0065
  ]
  edge [
    source 0
    target 43
    latency "85 ms"
    packet_loss 0.0197
  ]
  edge [
    source 0
    target 44
    latency "28 ms"
    packet_loss 0.01
  ]
  edge [
    source 0
    target 45
    latency "196 ms"
    packet_loss 0.033
  ]
  edge [
    source 0
    target 46
    latency "115 ms"
    packet_loss 0.0195
  ]
  edge [
    source 0
    target 47
    latency "298 ms"
    packet_loss 0.0417
  ]
  edge [
    source 0
    target 48
    latency "55 ms"
    packet_loss 0.0125
  ]
  edge [
    source 0
    target 49
    latency "158 ms"
    packet_loss 0.0486
  ]
  edge [
    source 1
    target 1
    latency "8 ms"
    packet_loss 0.04
  ]
  edge [
    source 1
    target 2
    latency "175 ms"
    packet_loss 0.0426
  ]
  edge [
    source 1
    target 3
    latency "149 ms"
    packet_loss 0.0453
  ]
  edge [
    source 1
    target 4
    latency "81 ms"
    packet_loss 0.0127
  ]
  edge [
    source 1
    target 5
    latency "168 ms"
    packet_loss 0.0341
  ]
  edge [
    source 1
    target 6
    latency "4 ms"
    packet_loss 0.0198
  ]
  edge [
    source 1
    target 7
    latency "187 ms"
    packet_loss 0.0347
  ]
  edge [
    source 1
    target 8
    latency "66 ms"
    packet_loss 0.0166
  ]
  edge [
    source 1
    target 9
    latency "163 ms"
    packet_loss 0.0474
  ]
  edge [
    source 1
    target 10
    latency "243 ms"
    packet_loss 0.0233
  ]
  edge [
    source 1
    target 11
    latency "202 ms"
    packet_loss 0.0212
  ]
  edge [
    source 1
    target 12
    latency "235 ms"
    packet_loss 0.0057
  ]
  edge [
    source 1
    target 13
    latency "282 ms"
    packet_loss 0.0404
  ]
  edge [
    source 1
    target 14
    latency "157 ms"
    packet_loss 0.0404
  ]
  edge [
    source 1
    target 15
    latency "117 ms"
    packet_loss 0.0295
  ]
  edge [
    source 1
    target 16
    latency "266 ms"
    packet_loss 0.0342
  ]
  edge [
    source 1
    target 17
    latency "294 ms"
    packet_loss 0.014
  ]
  edge [
    source 1
    target 18
    latency "241 ms"
    packet_loss 0.0094
  ]
  edge [
    source 1
    target 19
    latency "173 ms"
    packet_loss 0.0308
  ]
  edge [
    source 1
    target 20
    latency "12 ms"
    packet_loss 0.0325
  ]
  edge [
    source 1
    target 21
    latency "262 ms"
    packet_loss 0.0382
  ]
  edge [
    source 1
    target 22
    latency "270 ms"
    packet_loss 0.0205
  ]
  edge [
    source 1
    target 23
    latency "64 ms"
    packet_loss 0.0327
  ]
  edge [
    source 1
    target 24
    latency "145 ms"
    packet_loss 0.0177
  ]
  edge [
    source 1
    target 25
    latency "129 ms"
    packet_loss 0.0289
  ]
  edge [
    source 1
    target 26
    latency "228 ms"
    packet_loss 0.0139
  ]
  edge [
    source 1
    target 27
    latency "20 ms"
    packet_loss 0.0106
  ]
  edge [
    source 1
    target 28
    latency "85 ms"
    packet_loss 0.016
  ]
  edge [
    source 1
    target 29
    latency "118 ms"
    packet_loss 0.0088
  ]
  edge [
    source 1
    target 30
    latency "242 ms"
    packet_loss 0.0212
  ]
  edge [
    source 1
    target 31
    latency "180 ms"
    packet_loss 0.0337
  ]
  edge [
    source 1
    target 32
    latency "31 ms"
    packet_loss 0.0069
  ]
  edge [
    source 1
    target 33
    latency "25 ms"
    packet_loss 0.016
  ]
  edge [
    source 1
    target 34
    latency "21 ms"
    packet_loss 0.0118
  ]
  edge [
    source 1
    target 35
    latency "186 ms"
    packet_loss 0.0266
  ]
  edge [
    source 1
    target 36
    latency "141 ms"
    packet_loss 0.0178
  ]
  edge [
    source 1
    target 37
    latency "181 ms"
    packet_loss 0.0403
  ]
  edge [
    source 1
    target 38
    latency "230 ms"
    packet_loss 0.0198
  ]
  edge [
    source 1
    target 39
    latency "19 ms"
    packet_loss 0.0315
  ]
  edge [
    source 1
    target 40
    latency "162 ms"
    packet_loss 0.0333
  ]
  edge [
    source 1
    target 41
    latency "243 ms"
    packet_loss 0.0339
  ]
  edge [
    source 1
    target 42
    latency "281 ms"
    packet_loss 0.0294
  ]
  edge [
    source 1
    target 43
    latency "262 ms"
    packet_loss 0.0328
  ]
  edge [
    source 1
    target 44
    latency "161 ms"
    packet_loss 0.0201
  ]
  edge [
    source 1
    target 45
    latency "205 ms"
    packet_loss 0.0045
  ]
  edge [
    source 1
    target 46
    latency "295 ms"
    packet_loss 0.005
  ]
  edge [
    source 1
    target 47
    latency "177 ms"
    packet_loss 0.0263
  ]
  edge [
    source 1
    target 48
    latency "300 ms"
    packet_loss 0.004
  ]
  edge [
    source 1
    target 49
    latency "113 ms"
    packet_loss 0.0344
  ]
  edge [
    source 2
    target 2
    latency "3 ms"
    packet_loss 0.0457
  ]
  edge [
    source 2
    target 3
    latency "121 ms"
    packet_loss 0.0403
  ]
  edge [
    source 2
    target 4
    latency "154 ms"
    packet_loss 0.0455
  ]
  edge [
    source 2
    target 5
    latency "242 ms"
    packet_loss 0.0189
  ]
  edge [
    source 2
    target 6
    latency "138 ms"
    packet_loss 0.025
  ]
  edge [
    source 2
    target 7
    latency "210 ms"
    packet_loss 0.0041
  ]
  edge [
    source 2
    target 8
    latency "172 ms"
    packet_loss 0.0071
  ]
  edge [
    source 2
    target 9
    latency "55 ms"
    packet_loss 0.0493
  ]
  edge [
    source 2
    target 10
    latency "141 ms"
    packet_loss 0.0184
  ]
  edge [
    source 2
    target 11
    latency "74 ms"
    packet_loss 0.0263
  ]
  edge [
    source 2
    target 12
    latency "127 ms"
    packet_loss 0.0286
  ]
  edge [
    source 2
    target 13
    latency "280 ms"
    packet_loss 0.0264
  ]
  edge [
    source 2
    target 14
    latency "68 ms"
    packet_loss 0.0482
  ]
  edge [
    source 2
    target 15
    latency "10 ms"
    packet_loss 0.0026
  ]
  edge [
    source 2
    target 16
    latency "224 ms"
    packet_loss 0.0442
  ]
  edge [
    source 2
    target 17
    latency "95 ms"
    packet_loss 0.0213
  ]
  edge [
    source 2
    target 18
    latency "157 ms"
    packet_loss 0.0162
  ]
  edge [
    source 2
    target 19
    latency "124 ms"
    packet_loss 0.0353
  ]
  edge [
    source 2
    target 20
    latency "275 ms"
    packet_loss 0.0044
  ]
  edge [
    source 2
    target 21
    latency "33 ms"
    packet_loss 0.0241
  ]
  edge [
    source 2
    target 22
    latency "264 ms"
    packet_loss 0.0186
  ]
  edge [
    source 2
    target 23
    latency "281 ms"
    packet_loss 0.0139
  ]
  edge [
    source 2
    target 24
    latency "89 ms"
    packet_loss 0.024
  ]
  edge [
    source 2
    target 25
    latency "177 ms"
    packet_loss 0.0119
  ]
  edge [
    source 2
    target 26
    latency "176 ms"
    packet_loss 0.0094
  ]
  edge [
    source 2
    target 27
    latency "245 ms"
    packet_loss 0.001
  ]
  edge [
    source 2
    target 28
    latency "127 ms"
    packet_loss 0.0122
  ]
  edge [
    source 2
    target 29
    latency "124 ms"
    packet_loss 0.0295
  ]
  edge [
    source 2
    target 30
    latency "219 ms"
    packet_loss 0.0367
  ]
  edge [
    source 2
    target 31
    latency "296 ms"
    packet_loss 0.0169
  ]
  edge [
    source 2
    target 32
    latency "80 ms"
    packet_loss 0.0013
  ]
  edge [
    source 2
    target 33
    latency "165 ms"
    packet_loss 0.0149
  ]
  edge [
    source 2
    target 34
    latency "65 ms"
    packet_loss 0.0469
  ]
  edge [
    source 2
    target 35
    latency "218 ms"
    packet_loss 0.0019
  ]
  edge [
    source 2
    target 36
    latency "15 ms"
    packet_loss 0.0346
  ]
  edge [
    source 2
    target 37
    latency "122 ms"
    packet_loss 0.028
  ]
  edge [
    source 2
    target 38
    latency "106 ms"
    packet_loss 0.0478
  ]
  edge [
    source 2
    target 39
    latency "247 ms"
    packet_loss 0.002
  ]
  edge [
    source 2
    target 40
    latency "195 ms"
    packet_loss 0.0023
  ]
  edge [
    source 2
    target 41
    latency "222 ms"
    packet_loss 0.0239
  ]
  edge [
    source 2
    target 42
    latency "260 ms"
    packet_loss 0.0297
  ]
  edge [
    source 2
    target 43
    latency "242 ms"
    packet_loss 0.0122
  ]
  edge [
    source 2
    target 44
    latency "163 ms"
    packet_loss 0.0444
  ]
  edge [
    source 2
    target 45
    latency "28 ms"
    packet_loss 0.032
  ]
  edge [
    source 2
    target 46
    latency "118 ms"
    packet_loss 0.0335
  ]
  edge [
    source 2
    target 47
    latency "107 ms"
    packet_loss 0.0376
  ]
  edge [
    source 2
    target 48
    latency "231 ms"
    packet_loss 0.0364
  ]
  edge [
    source 2
    target 49
    latency "157 ms"
    packet_loss 0.0384
  ]
  edge [
    source 3
    target 3
    latency "8 ms"
    packet_loss 0.0497
  ]
  edge [
    source 3
    target 4
    latency "221 ms"
    packet_loss 0.0346
  ]
  edge [
    source 3
    target 5
    latency "251 ms"
    packet_loss 0.0298
  ]
  edge [
    source 3
    target 6
    latency "122 ms"
    packet_loss 0.004
  ]
  edge [
    source 3
    target 7
    latency "145 ms"
    packet_loss 0.0244
  ]
  edge [
    source 3
    target 8
    latency "171 ms"
    packet_loss 0.0285
  ]
  edge [
    source 3
    target 9
    latency "238 ms"
    packet_loss 0.0471
  ]
  edge [
    source 3
    target 10
    latency "80 ms"
    packet_loss 0.0164
  ]
  edge [
    source 3
    target 11
    latency "42 ms"
    packet_loss 0.0358
  ]
  edge [
    source 3
    target 12
    latency "277 ms"
    packet_loss 0.0174
  ]
  edge [
    source 3
    target 13
    latency "138 ms"
    packet_loss 0.0144
  ]
  edge [
    source 3
    target 14
    latency "26 ms"
    packet_loss 0.0061
  ]
  edge [
    source 3
    target 15
    latency "190 ms"
    packet_loss 0.0469
  ]
  edge [
    source 3
    target 16
    latency "188 ms"
    packet_loss 0.0492
  ]
  edge [
    source 3
    target 17
    latency "27 ms"
    packet_loss 0.0369
  ]
  edge [
    source 3
    target 18
    latency "130 ms"
    packet_loss 0.0237
  ]
  edge [
    source 3
    target 19
    latency "165 ms"
    packet_loss 0.0071
  ]
  edge [
    source 3
    target 20
    latency "30 ms"
    packet_loss 0.0208
  ]
  edge [
    source 3
    target 21
    latency "229 ms"
    packet_loss 0.0349
  ]
  edge [
    source 3
    target 22
    latency "270 ms"
    packet_loss 0.0461
  ]
  edge [
    source 3
    target 23
    latency "126 ms"
    packet_loss 0.0166
  ]
  edge [
    source 3
    target 24
    latency "251 ms"
    packet_loss 0.049
  ]
  edge [
    source 3
    target 25
    latency "296 ms"
    packet_loss 0.0378
  ]
  edge [
    source 3
    target 26
    latency "125 ms"
    packet_loss 0.0415
  ]
  edge [
    source 3
    target 27
    latency "156 ms"
    packet_loss 0.0055
  ]
  edge [
    source 3
    target 28
    latency "255 ms"
    packet_loss 0.0025
  ]
  edge [
    source 3
    target 29
    latency "29 ms"
    packet_loss 0.0127
  ]
  edge [
    source 3
    target 30
    latency "51 ms"
    packet_loss 0.0387
  ]
  edge [
    source 3
    target 31
    latency "251 ms"
    packet_loss 0.0477
  ]
  edge [
    source 3
    target 32
    latency "95 ms"
    packet_loss 0.0216
  ]
  edge [
    source 3
    target 33
    latency "259 ms"
    packet_loss 0.0398
  ]
  edge [
    source 3
    target 34
    latency "98 ms"
    packet_loss 0.003
  ]
  edge [
    source 3
    target 35
    latency "247 ms"
    packet_loss 0.0017
  ]
  edge [
    source 3
    target 36
    latency "89 ms"
    packet_loss 0.0338
  ]
  edge [
    source 3
    target 37
    latency "168 ms"
    packet_loss 0.0258
  ]
  edge [
    source 3
    target 38
    latency "261 ms"
    packet_loss 0.0426
  ]
  edge [
    source 3
    target 39
    latency "55 ms"
    packet_loss 0.0059
  ]
  edge [
    source 3
    target 40
    latency "262 ms"
    packet_loss 0.0035
  ]
  edge [
    source 3
    target 41
    latency "93 ms"
    packet_loss 0.014
  ]
  edge [
    source 3
    target 42
    latency "18 ms"
    packet_loss 0.0127
  ]
  edge [
    source 3
    target 43
    latency "237 ms"
    packet_loss 0.0439
  ]
  edge [
    source 3
    target 44
    latency "238 ms"
    packet_loss 0.0379
  ]
  edge [
    source 3
    target 45
    latency "250 ms"
    packet_loss 0.0223
  ]
  edge [
    source 3
    target 46
    latency "240 ms"
    packet_loss 0.0051
  ]
  edge [
    source 3
    target 47
    latency "124 ms"
    packet_loss 0.0461
  ]
  edge [
    source 3
    target 48
    latency "93 ms"
    packet_loss 0.018
  ]
  edge [
    source 3
    target 49
    latency "69 ms"
    packet_loss 0.0475
  ]
  edge [
    source 4
    target 4
    latency "1 ms"
    packet_loss 0.0439
  ]
  edge [
    source 4
    target 5
    latency "248 ms"
    packet_loss 0.0277
  ]
  edge [
    source 4
    target 6
    latency "164 ms"
    packet_loss 0.0438
  ]
  edge [
    source 4
    target 7
    latency "71 ms"
    packet_loss 0.0256
  ]
  edge [
    source 4
    target 8
    latency "15 ms"
    packet_loss 0.0099
  ]
  edge [
    source 4
    target 9
    latency "116 ms"
    packet_loss 0.0352
  ]
  edge [
    source 4
    target 10
    latency "232 ms"
    packet_loss 0.0307
  ]
  edge [
    source 4
    target 11
    latency "286 ms"
    packet_loss 0.047
  ]
  edge [
    source 4
    target 12
    latency "234 ms"
    packet_loss 0.017
  ]
  edge [
    source 4
    target 13
    latency "32 ms"
    packet_loss 0.0334
  ]
  edge [
    source 4
    target 14
    latency "300 ms"
    packet_loss 0.0138
  ]
  edge [
    source 4
    target 15
    latency "280 ms"
    packet_loss 0.0174
  ]
  edge [
    source 4
    target 16
    latency "230 ms"
    packet_loss 0.0471
  ]
  edge [
    source 4
    target 17
    latency "296 ms"
    packet_loss 0.0349
  ]
  edge [
    source 4
    target 18
    latency "96 ms"
    packet_loss 0.0326
  ]
  edge [
    source 4
    target 19
    latency "60 ms"
    packet_loss 0.0405
  ]
  edge [
    source 4
    target 20
    latency "25 ms"
    packet_loss 0.0442
  ]
  edge [
    source 4
    target 21
    latency "136 ms"
    packet_loss 0.0217
  ]
  edge [
    source 4
    target 22
    latency "57 ms"
    packet_loss 0.0415
  ]
  edge [
    source 4
    target 23
    latency "197 ms"
    packet_loss 0.011
  ]
  edge [
    source 4
    target 24
    latency "181 ms"
    packet_loss 0.0236
  ]
  edge [
    source 4
    target 25
    latency "259 ms"
    packet_loss 0.0062
  ]
  edge [
    source 4
    target 26
    latency "18 ms"
    packet_loss 0.0097
  ]
  edge [
    source 4
    target 27
    latency "300 ms"
    packet_loss 0.032
  ]
  edge [
    source 4
    target 28
    latency "152 ms"
    packet_loss 0.0368
  ]
  edge [
    source 4
    target 29
    latency "48 ms"
    packet_loss 0.0283
  ]
  edge [
    source 4
    target 30
    latency "112 ms"
    packet_loss 0.0208
  ]
  edge [
    source 4
    target 31
    latency "23 ms"
    packet_loss 0.0136
  ]
  edge [
    source 4
    target 32
    latency "142 ms"
    packet_loss 0.0211
  ]
  edge [
    source 4
    target 33
    latency "194 ms"
    packet_loss 0.037
  ]
  edge [
    source 4
    target 34
    latency "132 ms"
    packet_loss 0.0042
  ]
  edge [
    source 4
    target 35
    latency "225 ms"
    packet_loss 0.0195
  ]
  edge [
    source 4
    target 36
    latency "275 ms"
    packet_loss 0.0025
  ]
  edge [
    source 4
    target 37
    latency "31 ms"
    packet_loss 0.0432
  ]
  edge [
    source 4
    target 38
    latency "62 ms"
    packet_loss 0.0486
  ]
  edge [
    source 4
    target 39
    latency "182 ms"
    packet_loss 0.0454
  ]
  edge [
    source 4
    target 40
    latency "143 ms"
    packet_loss 0.0186
  ]
  edge [
    source 4
    target 41
    latency "269 ms"
    packet_loss 0.0315
  ]
  edge [
    source 4
    target 42
    latency "81 ms"
    packet_loss 0.0346
  ]
  edge [
    source 4
    target 43
    latency "128 ms"
    packet_loss 0.0488
  ]
  edge [
    source 4
    target 44
    latency "153 ms"
    packet_loss 0.0097
  ]
  edge [
    source 4
    target 45
    latency "294 ms"
    packet_loss 0.0399
  ]
  edge [
    source 4
    target 46
    latency "262 ms"
    packet_loss 0.0495
  ]
  edge [
    source 4
    target 47
    latency "121 ms"
    packet_loss 0.013
  ]
  edge [
    source 4
    target 48
    latency "78 ms"
    packet_loss 0.0029
  ]
  edge [
    source 4
    target 49
    latency "71 ms"
    packet_loss 0.0455
  ]
  edge [
    source 5
    target 5
    latency "9 ms"
    packet_loss 0.008
  ]
  edge [
    source 5
    target 6
    latency "125 ms"
    packet_loss 0.0117
  ]
  edge [
    source 5
    target 7
    latency "213 ms"
    packet_loss 0.0265
  ]
  edge [
    source 5
    target 8
    latency "254 ms"
    packet_loss 0.0442
  ]
  edge [
    source 5
    target 9
    latency "179 ms"
    packet_loss 0.0261
  ]
  edge [
    source 5
    target 10
    latency "111 ms"
    packet_loss 0.0178
  ]
  edge [
    source 5
    target 11
    latency "189 ms"
    packet_loss 0.0029
  ]
  edge [
    source 5
    target 12
    latency "194 ms"
    packet_loss 0.0184
  ]
  edge [
    source 5
    target 13
    latency "113 ms"
    packet_loss 0.0459
  ]
  edge [
    source 5
    target 14
    latency "33 ms"
    packet_loss 0.0236
  ]
  edge [
    source 5
    target 15
    latency "24 ms"
    packet_loss 0.0385
  ]
  edge [
    source 5
    target 16
    latency "261 ms"
    packet_loss 0.0035
  ]
  edge [
    source 5
    target 17
    latency "238 ms"
    packet_loss 0.0476
  ]
  edge [
    source 5
    target 18
    latency "143 ms"
    packet_loss 0.0204
  ]
  edge [
    source 5
    target 19
    latency "262 ms"
    packet_loss 0.0111
  ]
  edge [
    source 5
    target 20
    latency "115 ms"
    packet_loss 0.0314
  ]
  edge [
    source 5
    target 21
    latency "156 ms"
    packet_loss 0.0258
  ]
  edge [
    source 5
    target 22
    latency "117 ms"
    packet_loss 0.0074
  ]
  edge [
    source 5
    target 23
    latency "179 ms"
    packet_loss 0.0192
  ]
  edge [
    source 5
    target 24
    latency "198 ms"
    packet_loss 0.0142
  ]
  edge [
    source 5
    target 25
    latency "196 ms"
    packet_loss 0.0042
  ]
  edge [
    source 5
    target 26
    latency "134 ms"
    packet_loss 0.0354
  ]
  edge [
    source 5
    target 27
    latency "177 ms"
    packet_loss 0.0399
  ]
  edge [
    source 5
    target 28
    latency "181 ms"
    packet_loss 0.0259
  ]
  edge [
    source 5
    target 29
    latency "206 ms"
    packet_loss 0.0063
  ]
  edge [
    source 5
    target 30
    latency "69 ms"
    packet_loss 0.0073
  ]
  edge [
    source 5
    target 31
    latency "246 ms"
    packet_loss 0.017
  ]
  edge [
    source 5
    target 32
    latency "194 ms"
    packet_loss 0.0284
  ]
  edge [
    source 5
    target 33
    latency "50 ms"
    packet_loss 0.0435
  ]
  edge [
    source 5
    target 34
    latency "125 ms"
    packet_loss 0.0145
  ]
  edge [
    source 5
    target 35
    latency "152 ms"
    packet_loss 0.0142
  ]
  edge [
    source 5
    target 36
    latency "99 ms"
    packet_loss 0.0412
  ]
  edge [
    source 5
    target 37
    latency "261 ms"
    packet_loss 0.0174
  ]
  edge [
    source 5
    target 38
    latency "265 ms"
    packet_loss 0.0373
  ]
  edge [
    source 5
    target 39
    latency "4 ms"
    packet_loss 0.0105
  ]
  edge [
    source 5
    target 40
    latency "116 ms"
    packet_loss 0.0465
  ]
  edge [
    source 5
    target 41
    latency "6 ms"
    packet_loss 0.0217
  ]
  edge [
    source 5
    target 42
    latency "132 ms"
    packet_loss 0.007
  ]
  edge [
    source 5
    target 43
    latency "92 ms"
    packet_loss 0.0434
  ]
  edge [
    source 5
    target 44
    latency "38 ms"
    packet_loss 0.006
  ]
  edge [
    source 5
    target 45
    latency "217 ms"
    packet_loss 0.0464
  ]
  edge [
    source 5
    target 46
    latency "109 ms"
    packet_loss 0.0356
  ]
  edge [
    source 5
    target 47
    latency "111 ms"
    packet_loss 0.0181
  ]
  edge [
    source 5
    target 48
    latency "52 ms"
    packet_loss 0.0224
  ]
  edge [
    source 5
    target 49
    latency "121 ms"
    packet_loss 0.0472
  ]
  edge [
    source 6
    target 6
    latency "10 ms"
    packet_loss 0.0305
  ]
  edge [
    source 6
    target 7
    latency "87 ms"
    packet_loss 0.0254
  ]
  edge [
    source 6
    target 8
    latency "173 ms"
    packet_loss 0.0168
  ]
  edge [
    source 6
    target 9
    latency "229 ms"
    packet_loss 0.0246
  ]
  edge [
    source 6
    target 10
    latency "199 ms"
    packet_loss 0.0134
  ]
  edge [
    source 6
    target 11
    latency "205 ms"
    packet_loss 0.0428
  ]
  edge [
    source 6
    target 12
    latency "109 ms"
    packet_loss 0.0312
  ]
  edge [
    source 6
    target 13
    latency "38 ms"
    packet_loss 0.0362
  ]
  edge [
    source 6
    target 14
    latency "201 ms"
    packet_loss 0.0399
  ]
  edge [
    source 6
    target 15
    latency "217 ms"
    packet_loss 0.0438
  ]
  edge [
    source 6
    target 16
    latency "178 ms"
    packet_loss 0.0125
  ]
  edge [
    source 6
    target 17
    latency "191 ms"
    packet_loss 0.0438
  ]
  edge [
    source 6
    target 18
    latency "268 ms"
    packet_loss 0.0104
  ]
  edge [
    source 6
    target 19
    latency "200 ms"
    packet_loss 0.0395
  ]
  edge [
    source 6
    target 20
    latency "79 ms"
    packet_loss 0.0162
  ]
  edge [
    source 6
    target 21
    latency "131 ms"
    packet_loss 0.0288
  ]
  edge [
    source 6
    target 22
    latency "124 ms"
    packet_loss 0.0306
  ]
  edge [
    source 6
    target 23
    latency "254 ms"
    packet_loss 0.0344
  ]
  edge [
    source 6
    target 24
    latency "238 ms"
    packet_loss 0.0272
  ]
  edge [
    source 6
    target 25
    latency "275 ms"
    packet_loss 0.0143
  ]
  edge [
    source 6
    target 26
    latency "213 ms"
    packet_loss 0.0124
  ]
  edge [
    source 6
    target 27
    latency "162 ms"
    packet_loss 0.0016
  ]
  edge [
    source 6
    target 28
    latency "33 ms"
    packet_loss 0.0414
  ]
  edge [
    source 6
    target 29
    latency "9 ms"
    packet_loss 0.0438
  ]
  edge [
    source 6
    target 30
    latency "32 ms"
    packet_loss 0.0
  ]
  edge [
    source 6
    target 31
    latency "68 ms"
    packet_loss 0.0464
  ]
  edge [
    source 6
    target 32
    latency "212 ms"
    packet_loss 0.0299
  ]
  edge [
    source 6
    target 33
    latency "175 ms"
    packet_loss 0.0113
  ]
  edge [
    source 6
    target 34
    latency "5 ms"
    packet_loss 0.0074
  ]
  edge [
    source 6
    target 35
    latency "136 ms"
    packet_loss 0.0072
  ]
  edge [
    source 6
    target 36
    latency "221 ms"
    packet_loss 0.0377
  ]
  edge [
    source 6
    target 37
    latency "177 ms"
    packet_loss 0.0292
  ]
  edge [
    source 6
    target 38
    latency "244 ms"
    packet_loss 0.012
  ]
  edge [
    source 6
    target 39
    latency "290 ms"
    packet_loss 0.0016
  ]
  edge [
    source 6
    target 40
    latency "3 ms"
    packet_loss 0.015
  ]
  edge [
    source 6
    target 41
    latency "76 ms"
    packet_loss 0.0021
  ]
  edge [
    source 6
    target 42
    latency "166 ms"
    packet_loss 0.0183
  ]
  edge [
    source 6
    target 43
    latency "93 ms"
    packet_loss 0.0028
  ]
  edge [
    source 6
    target 44
    latency "168 ms"
    packet_loss 0.0291
  ]
  edge [
    source 6
    target 45
    latency "91 ms"
    packet_loss 0.0176
  ]
  edge [
    source 6
    target 46
    latency "282 ms"
    packet_loss 0.0306
  ]
  edge [
    source 6
    target 47
    latency "96 ms"
    packet_loss 0.0486
  ]
  edge [
    source 6
    target 48
    latency "179 ms"
    packet_loss 0.0373
  ]
  edge [
    source 6
    target 49
    latency "92 ms"
    packet_loss 0.0271
  ]
  edge [
    source 7
    target 7
    latency "3 ms"
    packet_loss 0.0054
  ]
  edge [
    source 7
    target 8
    latency "62 ms"
    packet_loss 0.0184
  ]
  edge [
    source 7
    target 9
    latency "60 ms"
    packet_loss 0.0403
  ]
  edge [
    source 7
    target 10
    latency "292 ms"
    packet_loss 0.0106
  ]
  edge [
    source 7
    target 11
    latency "129 ms"
    packet_loss 0.0438
  ]
  edge [
    source 7
    target 12
    latency "206 ms"
    packet_loss 0.0487
  ]
  edge [
    source 7
    target 13
    latency "194 ms"
    packet_loss 0.0487
  ]
  edge [
    source 7
    target 14
    latency "174 ms"
    packet_loss 0.006
  ]
  edge [
    source 7
    target 15
    latency "167 ms"
    packet_loss 0.0267
  ]
  edge [
    source 7
    target 16
    latency "146 ms"
    packet_loss 0.0029
  ]
  edge [
    source 7
    target 17
    latency "160 ms"
    packet_loss 0.0129
  ]
  edge [
    source 7
    target 18
    latency "80 ms"
    packet_loss 0.0439
  ]
  edge [
    source 7
    target 19
    latency "172 ms"
    packet_loss 0.0315
  ]
  edge [
    source 7
    target 20
    latency "277 ms"
    packet_loss 0.0458
  ]
  edge [
    source 7
    target 21
    latency "81 ms"
    packet_loss 0.0386
  ]
  edge [
    source 7
    target 22
    latency "213 ms"
    packet_loss 0.0096
  ]
  edge [
    source 7
    target 23
    latency "285 ms"
    packet_loss 0.0125
  ]
  edge [
    source 7
    target 24
    latency "22 ms"
    packet_loss 0.0493
  ]
  edge [
    source 7
    target 25
    latency "69 ms"
    packet_loss 0.006
  ]
  edge [
    source 7
    target 26
    latency "103 ms"
    packet_loss 0.0155
  ]
  edge [
    source 7
    target 27
    latency "290 ms"
    packet_loss 0.0045
  ]
  edge [
    source 7
    target 28
    latency "16 ms"
    packet_loss 0.0307
  ]
  edge [
    source 7
    target 29
    latency "77 ms"
    packet_loss 0.037
  ]
  edge [
    source 7
    target 30
    latency "4 ms"
    packet_loss 0.0222
  ]
  edge [
    source 7
    target 31
    latency "258 ms"
    packet_loss 0.0247
  ]
  edge [
    source 7
    target 32
    latency "254 ms"
    packet_loss 0.0267
  ]
  edge [
    source 7
    target 33
    latency "287 ms"
    packet_loss 0.0143
  ]
  edge [
    source 7
    target 34
    latency "213 ms"
    packet_loss 0.0232
  ]
  edge [
    source 7
    target 35
    latency "62 ms"
    packet_loss 0.0294
  ]
  edge [
    source 7
    target 36
    latency "160 ms"
    packet_loss 0.012
  ]
  edge [
    source 7
    target 37
    latency "118 ms"
    packet_loss 0.012
  ]
  edge [
    source 7
    target 38
    latency "29 ms"
    packet_loss 0.0455
  ]
  edge [
    source 7
    target 39
    latency "194 ms"
    packet_loss 0.0357
  ]
  edge [
    source 7
    target 40
    latency "141 ms"
    packet_loss 0.0262
  ]
  edge [
    source 7
    target 41
    latency "47 ms"
    packet_loss 0.0087
  ]
  edge [
    source 7
    target 42
    latency "70 ms"
    packet_loss 0.0186
  ]
  edge [
    source 7
    target 43
    latency "156 ms"
    packet_loss 0.0349
  ]
  edge [
    source 7
    target 44
    latency "139 ms"
    packet_loss 0.0137
  ]
  edge [
    source 7
    target 45
    latency "137 ms"
    packet_loss 0.0167
  ]
  edge [
    source 7
    target 46
    latency "82 ms"
    packet_loss 0.0292
  ]
  edge [
    source 7
    target 47
    latency "167 ms"
    packet_loss 0.004
  ]
  edge [
    source 7
    target 48
    latency "123 ms"
    packet_loss 0.0101
  ]
  edge [
    source 7
    target 49
    latency "62 ms"
    packet_loss 0.0131
  ]
  edge [
    source 8
    target 8
    latency "1 ms"
    packet_loss 0.0123
  ]
  edge [
    source 8
    target 9
    latency "277 ms"
    packet_loss 0.0474
  ]
  edge [
    source 8
    target 10
    latency "198 ms"
    packet_loss 0.0251
  ]
  edge [
    source 8
    target 11
    latency "29 ms"
    packet_loss 0.0443
  ]
  edge [
    source 8
    target 12
    latency "122 ms"
    packet_loss 0.0299
  ]
  edge [
    source 8
    target 13
    latency "38 ms"
    packet_loss 0.028
  ]
  edge [
    source 8
    target 14
    latency "213 ms"
    packet_loss 0.0394
  ]
  edge [
    source 8
    target 15
    latency "241 ms"
    packet_loss 0.0325
  ]
  edge [
    source 8
    target 16
    latency "171 ms"
    packet_loss 0.0039
  ]
  edge [
    source 8
    target 17
    latency "82 ms"
    packet_loss 0.0231
  ]
  edge [
    source 8
    target 18
    latency "118 ms"
    packet_loss 0.0015
  ]
  edge [
    source 8
    target 19
    latency "110 ms"
    packet_loss 0.0331
  ]
  edge [
    source 8
    target 20
    latency "26 ms"
    packet_loss 0.0256
  ]
  edge [
    source 8
    target 21
    latency "97 ms"
    packet_loss 0.0138
  ]
  edge [
    source 8
    target 22
    latency "74 ms"
    packet_loss 0.0001
  ]
  edge [
    source 8
    target 23
    latency "24 ms"
    packet_loss 0.0114
  ]
  edge [
    source 8
    target 24
    latency "146 ms"
    packet_loss 0.0067
  ]
  edge [
    source 8
    target 25
    latency "10 ms"
    packet_loss 0.0064
  ]
  edge [
    source 8
    target 26
    latency "227 ms"
    packet_loss 0.0192
  ]
  edge [
    source 8
    target 27
    latency "252 ms"
    packet_loss 0.0041
  ]
  edge [
    source 8
    target 28
    latency "72 ms"
    packet_loss 0.0192
  ]
  edge [
    source 8
    target 29
    latency "288 ms"
    packet_loss 0.0112
  ]
  edge [
    source 8
    target 30
    latency "83 ms"
    packet_loss 0.0478
  ]
  edge [
    source 8
    target 31
    latency "3 ms"
    packet_loss 0.0394
  ]
  edge [
    source 8
    target 32
    latency "67 ms"
    packet_loss 0.0247
  ]
  edge [
    source 8
    target 33
    latency "87 ms"
    packet_loss 0.0387
  ]
  edge [
    source 8
    target 34
    latency "262 ms"
    packet_loss 0.025
  ]
  edge [
    source 8
    target 35
    latency "52 ms"
    packet_loss 0.0454
  ]
  edge [
    source 8
    target 36
    latency "178 ms"
    packet_loss 0.007
  ]
  edge [
    source 8
    target 37
    latency "86 ms"
    packet_loss 0.0447
  ]
  edge [
    source 8
    target 38
    latency "201 ms"
    packet_loss 0.0006
  ]
  edge [
    source 8
    target 39
    latency "174 ms"
    packet_loss 0.0452
  ]
  edge [
    source 8
    target 40
    latency "110 ms"
    packet_loss 0.0226
  ]
  edge [
    source 8
    target 41
    latency "174 ms"
    packet_loss 0.0293
  ]
  edge [
    source 8
    target 42
    latency "94 ms"
    packet_loss 0.0456
  ]
  edge [
    source 8
    target 43
    latency "121 ms"
    packet_loss 0.0099
  ]
  edge [
    source 8
    target 44
    latency "242 ms"
    packet_loss 0.0478
  ]
  edge [
    source 8
    target 45
    latency "261 ms"
    packet_loss 0.0182
  ]
  edge [
    source 8
    target 46
    latency "194 ms"
    packet_loss 0.0081
  ]
  edge [
    source 8
    target 47
    latency "246 ms"
    packet_loss 0.0156
  ]
  edge [
    source 8
    target 48
    latency "17 ms"
    packet_loss 0.0415
  ]
  edge [
    source 8
    target 49
    latency "114 ms"
    packet_loss 0.0357
  ]
  edge [
    source 9
    target 9
    latency "8 ms"
    packet_loss 0.0044
  ]
  edge [
    source 9
    target 10
    latency "110 ms"
    packet_loss 0.0199
  ]
  edge [
    source 9
    target 11
    latency "98 ms"
    packet_loss 0.0179
  ]
  edge [
    source 9
    target 12
    latency "219 ms"
    packet_loss 0.0455
  ]
  edge [
    source 9
    target 13
    latency "82 ms"
    packet_loss 0.0169
  ]
  edge [
    source 9
    target 14
    latency "218 ms"
    packet_loss 0.021
  ]
  edge [
    source 9
    target 15
    latency "283 ms"
    packet_loss 0.023
  ]
  edge [
    source 9
    target 16
    latency "18 ms"
    packet_loss 0.0405
  ]
  edge [
    source 9
    target 17
    latency "149 ms"
    packet_loss 0.0377
  ]
  edge [
    source 9
    target 18
    latency "15 ms"
    packet_loss 0.0221
  ]
  edge [
    source 9
    target 19
    latency "43 ms"
    packet_loss 0.0443
  ]
  edge [
    source 9
    target 20
    latency "177 ms"
    packet_loss 0.0425
  ]
  edge [
    source 9
    target 21
    latency "249 ms"
    packet_loss 0.0151
  ]
  edge [
    source 9
    target 22
    latency "262 ms"
    packet_loss 0.0305
  ]
  edge [
    source 9
    target 23
    latency "100 ms"
    packet_loss 0.0477
  ]
  edge [
    source 9
    target 24
    latency "135 ms"
    packet_loss 0.0495
  ]
  edge [
    source 9
    target 25
    latency "238 ms"
    packet_loss 0.0029
  ]
  edge [
    source 9
    target 26
    latency "165 ms"
    packet_loss 0.0132
  ]
  edge [
    source 9
    target 27
    latency "197 ms"
    packet_loss 0.0107
  ]
  edge [
    source 9
    target 28
    latency "232 ms"
    packet_loss 0.027
  ]
  edge [
    source 9
    target 29
    latency "29 ms"
    packet_loss 0.0474
  ]
  edge [
    source 9
    target 30
    latency "291 ms"
    packet_loss 0.0368
  ]
  edge [
    source 9
    target 31
    latency "48 ms"
    packet_loss 0.0103
  ]
  edge [
    source 9
    target 32
    latency "10 ms"
    packet_loss 0.0465
  ]
  edge [
    source 9
    target 33
    latency "38 ms"
    packet_loss 0.0444
  ]
  edge [
    source 9
    target 34
    latency "299 ms"
    packet_loss 0.0325
  ]
  edge [
    source 9
    target 35
    latency "60 ms"
    packet_loss 0.0332
  ]
  edge [
    source 9
    target 36
    latency "62 ms"
    packet_loss 0.0402
  ]
  edge [
    source 9
    target 37
    latency "156 ms"
    packet_loss 0.004
  ]
  edge [
    source 9
    target 38
    latency "99 ms"
    packet_loss 0.0199
  ]
  edge [
    source 9
    target 39
    latency "161 ms"
    packet_loss 0.0423
  ]
  edge [
    source 9
    target 40
    latency "86 ms"
    packet_loss 0.0473
  ]
  edge [
    source 9
    target 41
    latency "251 ms"
    packet_loss 0.0127
  ]
  edge [
    source 9
    target 42
    latency "200 ms"
    packet_loss 0.0131
  ]
  edge [
    source 9
    target 43
    latency "190 ms"
    packet_loss 0.0036
  ]
  edge [
    source 9
    target 44
    latency "299 ms"
    packet_loss 0.0477
  ]
  edge [
    source 9
    target 45
    latency "183 ms"
    packet_loss 0.0424
  ]
  edge [
    source 9
    target 46
    latency "67 ms"
    packet_loss 0.0344
  ]
  edge [
    source 9
    target 47
    latency "68 ms"
    packet_loss 0.0014
  ]
  edge [
    source 9
    target 48
    latency "232 ms"
    packet_loss 0.0375
  ]
  edge [
    source 9
    target 49
    latency "56 ms"
    packet_loss 0.0179
  ]
  edge [
    source 10
    target 10
    latency "5 ms"
    packet_loss 0.028
  ]
  edge [
    source 10
    target 11
    latency "184 ms"
    packet_loss 0.0334
  ]
  edge [
    source 10
    target 12
    latency "141 ms"
    packet_loss 0.0396
  ]
  edge [
    source 10
    target 13
    latency "24 ms"
    packet_loss 0.0321
  ]
  edge [
    source 10
    target 14
    latency "280 ms"
    packet_loss 0.0196
  ]
  edge [
    source 10
    target 15
    latency "253 ms"
    packet_loss 0.0066
  ]
  edge [
    source 10
    target 16
    latency "8 ms"
    packet_loss 0.0038
  ]
  edge [
    source 10
    target 17
    latency "168 ms"
    packet_loss 0.0344
  ]
  edge [
    source 10
    target 18
    latency "85 ms"
    packet_loss 0.0311
  ]
  edge [
    source 10
    target 19
    latency "187 ms"
    packet_loss 0.0485
  ]
  edge [
    source 10
    target 20
    latency "27 ms"
    packet_loss 0.0109
  ]
  edge [
    source 10
    target 21
    latency "6 ms"
    packet_loss 0.0132
  ]
  edge [
    source 10
    target 22
    latency "3 ms"
    packet_loss 0.0067
  ]
  edge [
    source 10
    target 23
    latency "12 ms"
    packet_loss 0.0176
  ]
  edge [
    source 10
    target 24
    latency "268 ms"
    packet_loss 0.0199
  ]
  edge [
    source 10
    target 25
    latency "10 ms"
    packet_loss 0.0089
  ]
  edge [
    source 10
    target 26
    latency "229 ms"
    packet_loss 0.0496
  ]
  edge [
    source 10
    target 27
    latency "223 ms"
    packet_loss 0.0193
  ]
  edge [
    source 10
    target 28
    latency "239 ms"
    packet_loss 0.0411
  ]
  edge [
    source 10
    target 29
    latency "195 ms"
    packet_loss 0.0016
  ]
  edge [
    source 10
    target 30
    latency "230 ms"
    packet_loss 0.0231
  ]
  edge [
    source 10
    target 31
    latency "300 ms"
    packet_loss 0.0271
  ]
  edge [
    source 10
    target 32
    latency "169 ms"
    packet_loss 0.0117
  ]
  edge [
    source 10
    target 33
    latency "203 ms"
    packet_loss 0.04
  ]
  edge [
    source 10
    target 34
    latency "246 ms"
    packet_loss 0.0312
  ]
  edge [
    source 10
    target 35
    latency "196 ms"
    packet_loss 0.002
  ]
  edge [
    source 10
    target 36
    latency "129 ms"
    packet_loss 0.0252
  ]
  edge [
    source 10
    target 37
    latency "296 ms"
    packet_loss 0.0246
  ]
  edge [
    source 10
    target 38
    latency "209 ms"
    packet_loss 0.002
  ]
  edge [
    source 10
    target 39
    latency "58 ms"
    packet_loss 0.0277
  ]
  edge [
    source 10
    target 40
    latency "37 ms"
    packet_loss 0.0406
  ]
  edge [
    source 10
    target 41
    latency "79 ms"
    packet_loss 0.0102
  ]
  edge [
    source 10
    target 42
    latency "299 ms"
    packet_loss 0.0108
  ]
  edge [
    source 10
    target 43
    latency "223 ms"
    packet_loss 0.0139
  ]
  edge [
    source 10
    target 44
    latency "51 ms"
    packet_loss 0.0213
  ]
  edge [
    source 10
    target 45
    latency "104 ms"
    packet_loss 0.0332
  ]
  edge [
    source 10
    target 46
    latency "260 ms"
    packet_loss 0.0168
  ]
  edge [
    source 10
    target 47
    latency "70 ms"
    packet_loss 0.0438
  ]
  edge [
    source 10
    target 48
    latency "41 ms"
    packet_loss 0.0156
  ]
  edge [
    source 10
    target 49
    latency "65 ms"
    packet_loss 0.0133
  ]
  edge [
    source 11
    target 11
    latency "10 ms"
    packet_loss 0.0285
  ]
  edge [
    source 11
    target 12
    latency "5 ms"
    packet_loss 0.0104
  ]
  edge [
    source 11
    target 13
    latency "280 ms"
    packet_loss 0.044
  ]
  edge [
    source 11
    target 14
    latency "234 ms"
    packet_loss 0.0066
  ]
  edge [
    source 11
    target 15
    latency "57 ms"
    packet_loss 0.0088
  ]
  edge [
    source 11
    target 16
    latency "139 ms"
    packet_loss 0.0154
  ]
  edge [
    source 11
    target 17
    latency "249 ms"
    packet_loss 0.0368
  ]
  edge [
    source 11
    target 18
    latency "29 ms"
    packet_loss 0.0323
  ]
  edge [
    source 11
    target 19
    latency "284 ms"
    packet_loss 0.021
  ]
  edge [
    source 11
    target 20
    latency "168 ms"
    packet_loss 0.0027
  ]
  edge [
    source 11
    target 21
    latency "181 ms"
    packet_loss 0.0227
  ]
  edge [
    source 11
    target 22
    latency "284 ms"
    packet_loss 0.0196
  ]
  edge [
    source 11
    target 23
    latency "72 ms"
    packet_loss 0.0294
  ]
  edge [
    source 11
    target 24
    latency "216 ms"
    packet_loss 0.0106
  ]
  edge [
    source 11
    target 25
    latency "246 ms"
    packet_loss 0.0404
  ]
  edge [
    source 11
    target 26
    latency "209 ms"
    packet_loss 0.0055
  ]
  edge [
    source 11
    target 27
    latency "12 ms"
    packet_loss 0.0252
  ]
  edge [
    source 11
    target 28
    latency "126 ms"
    packet_loss 0.0281
  ]
  edge [
    source 11
    target 29
    latency "80 ms"
    packet_loss 0.0281
  ]
  edge [
    source 11
    target 30
    latency "236 ms"
    packet_loss 0.0388
  ]
  edge [
    source 11
    target 31
    latency "36 ms"
    packet_loss 0.0468
  ]
  edge [
    source 11
    target 32
    latency "172 ms"
    packet_loss 0.0296
  ]
  edge [
    source 11
    target 33
    latency "137 ms"
    packet_loss 0.0497
  ]
  edge [
    source 11
    target 34
    latency "50 ms"
    packet_loss 0.0457
  ]
  edge [
    source 11
    target 35
    latency "130 ms"
    packet_loss 0.0463
  ]
  edge [
    source 11
    target 36
    latency "53 ms"
    packet_loss 0.0035
  ]
  edge [
    source 11
    target 37
    latency "266 ms"
    packet_loss 0.0211
  ]
  edge [
    source 11
    target 38
    latency "276 ms"
    packet_loss 0.0324
  ]
  edge [
    source 11
    target 39
    latency "254 ms"
    packet_loss 0.0489
  ]
  edge [
    source 11
    target 40
    latency "232 ms"
    packet_loss 0.0019
  ]
  edge [
    source 11
    target 41
    latency "259 ms"
    packet_loss 0.0301
  ]
  edge [
    source 11
    target 42
    latency "142 ms"
    packet_loss 0.0484
  ]
  edge [
    source 11
    target 43
    latency "241 ms"
    packet_loss 0.0431
  ]
  edge [
    source 11
    target 44
    latency "204 ms"
    packet_loss 0.0428
  ]
  edge [
    source 11
    target 45
    latency "120 ms"
    packet_loss 0.0341
  ]
  edge [
    source 11
    target 46
    latency "34 ms"
    packet_loss 0.0421
  ]
  edge [
    source 11
    target 47
    latency "280 ms"
    packet_loss 0.0209
  ]
  edge [
    source 11
    target 48
    latency "150 ms"
    packet_loss 0.0295
  ]
  edge [
    source 11
    target 49
    latency "261 ms"
    packet_loss 0.0143
  ]
  edge [
    source 12
    target 12
    latency "7 ms"
    packet_loss 0.0256
  ]
  edge [
    source 12
    target 13
    latency "192 ms"
    packet_loss 0.0357
  ]
  edge [
    source 12
    target 14
    latency "283 ms"
    packet_loss 0.0462
  ]
  edge [
    source 12
    target 15
    latency "5 ms"
    packet_loss 0.0178
  ]
  edge [
    source 12
    target 16
    latency "138 ms"
    packet_loss 0.0322
  ]
  edge [
    source 12
    target 17
    latency "121 ms"
    packet_loss 0.0393
  ]
  edge [
    source 12
    target 18
    latency "42 ms"
    packet_loss 0.0286
  ]
  edge [
    source 12
    target 19
    latency "154 ms"
    packet_loss 0.0149
  ]
  edge [
    source 12
    target 20
    latency "4 ms"
    packet_loss 0.0467
  ]
  edge [
    source 12
    target 21
    latency "53 ms"
    packet_loss 0.0373
  ]
  edge [
    source 12
    target 22
    latency "280 ms"
    packet_loss 0.0398
  ]
  edge [
    source 12
    target 23
    latency "152 ms"
    packet_loss 0.0101
  ]
  edge [
    source 12
    target 24
    latency "122 ms"
    packet_loss 0.0041
  ]
  edge [
    source 12
    target 25
    latency "250 ms"
    packet_loss 0.0187
  ]
  edge [
    source 12
    target 26
    latency "116 ms"
    packet_loss 0.0007
  ]
  edge [
    source 12
    target 27
    latency "92 ms"
    packet_loss 0.0319
  ]
  edge [
    source 12
    target 28
    latency "206 ms"
    packet_loss 0.0371
  ]
  edge [
    source 12
    target 29
    latency "30 ms"
    packet_loss 0.0312
  ]
  edge [
    source 12
    target 30
    latency "273 ms"
    packet_loss 0.0094
  ]
  edge [
    source 12
    target 31
    latency "89 ms"
    packet_loss 0.022
  ]
  edge [
    source 12
    target 32
    latency "18 ms"
    packet_loss 0.0229
  ]
  edge [
    source 12
    target 33
    latency "29 ms"
    packet_loss 0.0382
  ]
  edge [
    source 12
    target 34
    latency "141 ms"
    packet_loss 0.0236
  ]
  edge [
    source 12
    target 35
    latency "127 ms"
    packet_loss 0.0336
  ]
  edge [
    source 12
    target 36
    latency "19 ms"
    packet_loss 0.0348
  ]
  edge [
    source 12
    target 37
    latency "268 ms"
    packet_loss 0.0307
  ]
  edge [
    source 12
    target 38
    latency "129 ms"
    packet_loss 0.0279
  ]
  edge [
    source 12
    target 39
    latency "257 ms"
    packet_loss 0.0115
  ]
  edge [
    source 12
    target 40
    latency "13 ms"
    packet_loss 0.0173
  ]
  edge [
    source 12
    target 41
    latency "72 ms"
    packet_loss 0.0045
  ]
  edge [
    source 12
    target 42
    latency "153 ms"
    packet_loss 0.0479
  ]
  edge [
    source 12
    target 43
    latency "86 ms"
    packet_loss 0.0439
  ]
  edge [
    source 12
    target 44
    latency "69 ms"
    packet_loss 0.0267
  ]
  edge [
    source 12
    target 45
    latency "13 ms"
    packet_loss 0.0301
  ]
  edge [
    source 12
    target 46
    latency "219 ms"
    packet_loss 0.0046
  ]
  edge [
    source 12
    target 47
    latency "8 ms"
    packet_loss 0.0302
  ]
  edge [
    source 12
    target 48
    latency "7 ms"
    packet_loss 0.0024
  ]
  edge [
    source 12
    target 49
    latency "255 ms"
    packet_loss 0.0257
  ]
  edge [
    source 13
    target 13
    latency "1 ms"
    packet_loss 0.0102
  ]
  edge [
    source 13
    target 14
    latency "58 ms"
    packet_loss 0.0081
  ]
  edge [
    source 13
    target 15
    latency "228 ms"
    packet_loss 0.0247
  ]
  edge [
    source 13
    target 16
    latency "194 ms"
    packet_loss 0.0274
  ]
  edge [
    source 13
    target 17
    latency "103 ms"
    packet_loss 0.0188
  ]
  edge [
    source 13
    target 18
    latency "26 ms"
    packet_loss 0.0309
  ]
  edge [
    source 13
    target 19
    latency "290 ms"
    packet_loss 0.0027
  ]
  edge [
    source 13
    target 20
    latency "117 ms"
    packet_loss 0.0331
  ]
  edge [
    source 13
    target 21
    latency "277 ms"
    packet_loss 0.0137
  ]
  edge [
    source 13
    target 22
    latency "179 ms"
    packet_loss 0.0369
  ]
  edge [
    source 13
    target 23
    latency "5 ms"
    packet_loss 0.0319
  ]
  edge [
    source 13
    target 24
    latency "169 ms"
    packet_loss 0.0001
  ]
  edge [
    source 13
    target 25
    latency "19 ms"
    packet_loss 0.0491
  ]
  edge [
    source 13
    target 26
    latency "71 ms"
    packet_loss 0.0369
  ]
  edge [
    source 13
    target 27
    latency "154 ms"
    packet_loss 0.0152
  ]
  edge [
    source 13
    target 28
    latency "243 ms"
    packet_loss 0.0006
  ]
  edge [
    source 13
    target 29
    latency "128 ms"
    packet_loss 0.022
  ]
  edge [
    source 13
    target 30
    latency "71 ms"
    packet_loss 0.0097
  ]
  edge [
    source 13
    target 31
    latency "201 ms"
    packet_loss 0.0466
  ]
  edge [
    source 13
    target 32
    latency "116 ms"
    packet_loss 0.006
  ]
  edge [
    source 13
    target 33
    latency "166 ms"
    packet_loss 0.0333
  ]
  edge [
    source 13
    target 34
    latency "106 ms"
    packet_loss 0.0225
  ]
  edge [
    source 13
    target 35
    latency "28 ms"
    packet_loss 0.0039
  ]
  edge [
    source 13
    target 36
    latency "15 ms"
    packet_loss 0.0268
  ]
  edge [
    source 13
    target 37
    latency "51 ms"
    packet_loss 0.0003
  ]
  edge [
    source 13
    target 38
    latency "190 ms"
    packet_loss 0.021
  ]
  edge [
    source 13
    target 39
    latency "14 ms"
    packet_loss 0.0021
  ]
  edge [
    source 13
    target 40
    latency "84 ms"
    packet_loss 0.0269
  ]
  edge [
    source 13
    target 41
    latency "149 ms"
    packet_loss 0.0232
  ]
  edge [
    source 13
    target 42
    latency "198 ms"
    packet_loss 0.0152
  ]
  edge [
    source 13
    target 43
    latency "120 ms"
    packet_loss 0.047
  ]
  edge [
    source 13
    target 44
    latency "4 ms"
    packet_loss 0.0307
  ]
  edge [
    source 13
    target 45
    latency "250 ms"
    packet_loss 0.0022
  ]
  edge [
    source 13
    target 46
    latency "205 ms"
    packet_loss 0.0253
  ]
  edge [
    source 13
    target 47
    latency "24 ms"
    packet_loss 0.0405
  ]
  edge [
    source 13
    target 48
    latency "97 ms"
    packet_loss 0.0249
  ]
  edge [
    source 13
    target 49
    latency "122 ms"
    packet_loss 0.0006
  ]
  edge [
    source 14
    target 14
    latency "1 ms"
    packet_loss 0.025
  ]
  edge [
    source 14
    target 15
    latency "19 ms"
    packet_loss 0.036
  ]
  edge [
    source 14
    target 16
    latency "299 ms"
    packet_loss 0.0003
  ]
  edge [
    source 14
    target 17
    latency "237 ms"
    packet_loss 0.0277
  ]
  edge [
    source 14
    target 18
    latency "38 ms"
    packet_loss 0.027
  ]
  edge [
    source 14
    target 19
    latency "254 ms"
    packet_loss 0.0023
  ]
  edge [
    source 14
    target 20
    latency "293 ms"
    packet_loss 0.0269
  ]
  edge [
    source 14
    target 21
    latency "249 ms"
    packet_loss 0.0299
  ]
  edge [
    source 14
    target 22
    latency "201 ms"
    packet_loss 0.0283
  ]
  edge [
    source 14
    target 23
    latency "261 ms"
    packet_loss 0.0252
  ]
  edge [
    source 14
    target 24
    latency "86 ms"
    packet_loss 0.0082
  ]
  edge [
    source 14
    target 25
    latency "112 ms"
    packet_loss 0.0356
  ]
  edge [
    source 14
    target 26
    latency "63 ms"
    packet_loss 0.0435
  ]
  edge [
    source 14
    target 27
    latency "51 ms"
    packet_loss 0.0091
  ]
  edge [
    source 14
    target 28
    latency "24 ms"
    packet_loss 0.0208
  ]
  edge [
    source 14
    target 29
    latency "264 ms"
    packet_loss 0.0278
  ]
  edge [
    source 14
    target 30
    latency "109 ms"
    packet_loss 0.0461
  ]
  edge [
    source 14
    target 31
    latency "8 ms"
    packet_loss 0.0296
  ]
  edge [
    source 14
    target 32
    latency "192 ms"
    packet_loss 0.0409
  ]
  edge [
    source 14
    target 33
    latency "40 ms"
    packet_loss 0.0031
  ]
  edge [
    source 14
    target 34
    latency "138 ms"
    packet_loss 0.017
  ]
  edge [
    source 14
    target 35
    latency "223 ms"
    packet_loss 0.0469
  ]
  edge [
    source 14
    target 36
    latency "108 ms"
    packet_loss 0.0009
  ]
  edge [
    source 14
    target 37
    latency "14 ms"
    packet_loss 0.0055
  ]
  edge [
    source 14
    target 38
    latency "292 ms"
    packet_loss 0.0309
  ]
  edge [
    source 14
    target 39
    latency "179 ms"
    packet_loss 0.0423
  ]
  edge [
    source 14
    target 40
    latency "292 ms"
    packet_loss 0.0239
  ]
  edge [
    source 14
    target 41
    latency "247 ms"
    packet_loss 0.0047
  ]
  edge [
    source 14
    target 42
    latency "189 ms"
    packet_loss 0.0207
  ]
  edge [
    source 14
    target 43
    latency "114 ms"
    packet_loss 0.0037
  ]
  edge [
    source 14
    target 44
    latency "52 ms"
    packet_loss 0.0365
  ]
  edge [
    source 14
    target 45
    latency "128 ms"
    packet_loss 0.0248
  ]
  edge [
    source 14
    target 46
    latency "40 ms"
    packet_loss 0.003
  ]
  edge [
    source 14
    target 47
    latency "231 ms"
    packet_loss 0.026
  ]
  edge [
    source 14
    target 48
    latency "146 ms"
    packet_loss 0.0124
  ]
  edge [
    source 14
    target 49
    latency "267 ms"
    packet_loss 0.0446
  ]
  edge [
    source 15
    target 15
    latency "2 ms"
    packet_loss 0.0132
  ]
  edge [
    source 15
    target 16
    latency "266 ms"
    packet_loss 0.0214
  ]
  edge [
    source 15
    target 17
    latency "100 ms"
    packet_loss 0.0399
  ]
  edge [
    source 15
    target 18
    latency "118 ms"
    packet_loss 0.0058
  ]
  edge [
    source 15
    target 19
    latency "155 ms"
    packet_loss 0.0447
  ]
  edge [
    source 15
    target 20
    latency "233 ms"
    packet_loss 0.0342
  ]
  edge [
    source 15
    target 21
    latency "7 ms"
    packet_loss 0.0389
  ]
  edge [
    source 15
    target 22
    latency "199 ms"
    packet_loss 0.037
  ]
  edge [
    source 15
    target 23
    latency "101 ms"
    packet_loss 0.0004
  ]
  edge [
    source 15
    target 24
    latency "212 ms"
    packet_loss 0.0288
  ]
  edge [
    source 15
    target 25
    latency "24 ms"
    packet_loss 0.0174
  ]
  edge [
    source 15
    target 26
    latency "37 ms"
    packet_loss 0.0494
  ]
  edge [
    source 15
    target 27
    latency "278 ms"
    packet_loss 0.0309
  ]
  edge [
    source 15
    target 28
    latency "8 ms"
    packet_loss 0.0061
  ]
  edge [
    source 15
    target 29
    latency "16 ms"
    packet_loss 0.0252
  ]
  edge [
    source 15
    target 30
    latency "135 ms"
    packet_loss 0.0221
  ]
  edge [
    source 15
    target 31
    latency "218 ms"
    packet_loss 0.0251
  ]
  edge [
    source 15
    target 32
    latency "39 ms"
    packet_loss 0.0113
  ]
  edge [
    source 15
    target 33
    latency "54 ms"
    packet_loss 0.0098
  ]
  edge [
    source 15
    target 34
    latency "245 ms"
    packet_loss 0.0239
  ]
  edge [
    source 15
    target 35
    latency "244 ms"
    packet_loss 0.0217
  ]
  edge [
    source 15
    target 36
    latency "298 ms"
    packet_loss 0.0338
  ]
  edge [
    source 15
    target 37
    latency "236 ms"
    packet_loss 0.0131
  ]
  edge [
    source 15
    target 38
    latency "116 ms"
    packet_loss 0.0022
  ]
  edge [
    source 15
    target 39
    latency "103 ms"
    packet_loss 0.0005
  ]
  edge [
    source 15
    target 40
    latency "113 ms"
    packet_loss 0.0383
  ]
  edge [
    source 15
    target 41
    latency "70 ms"
    packet_loss 0.0179
  ]
  edge [
    source 15
    target 42
    latency "298 ms"
    packet_loss 0.0235
  ]
  edge [
    source 15
    target 43
    latency "75 ms"
    packet_loss 0.0015
  ]
  edge [
    source 15
    target 44
    latency "32 ms"
    packet_loss 0.0063
  ]
  edge [
    source 15
    target 45
    latency "234 ms"
    packet_loss 0.032
  ]
  edge [
    source 15
    target 46
    latency "33 ms"
    packet_loss 0.0334
  ]
  edge [
    source 15
    target 47
    latency "17 ms"
    packet_loss 0.037
  ]
  edge [
    source 15
    target 48
    latency "3 ms"
    packet_loss 0.0498
  ]
  edge [
    source 15
    target 49
    latency "58 ms"
    packet_loss 0.045
  ]
  edge [
    source 16
    target 16
    latency "9 ms"
    packet_loss 0.0481
  ]
  edge [
    source 16
    target 17
    latency "189 ms"
    packet_loss 0.0186
  ]
  edge [
    source 16
    target 18
    latency "244 ms"
    packet_loss 0.0148
  ]
  edge [
    source 16
    target 19
    latency "130 ms"
    packet_loss 0.0499
  ]
  edge [
    source 16
    target 20
    latency "262 ms"
    packet_loss 0.0398
  ]
  edge [
    source 16
    target 21
    latency "163 ms"
    packet_loss 0.0279
  ]
  edge [
    source 16
    target 22
    latency "222 ms"
    packet_loss 0.016
  ]
  edge [
    source 16
    target 23
    latency "266 ms"
    packet_loss 0.0307
  ]
  edge [
    source 16
    target 24
    latency "184 ms"
    packet_loss 0.0473
  ]
  edge [
    source 16
    target 25
    latency "269 ms"
    packet_loss 0.0404
  ]
  edge [
    source 16
    target 26
    latency "168 ms"
    packet_loss 0.0191
  ]
  edge [
    source 16
    target 27
    latency "1 ms"
    packet_loss 0.0269
  ]
  edge [
    source 16
    target 28
    latency "135 ms"
    packet_loss 0.0485
  ]
  edge [
    source 16
    target 29
    latency "104 ms"
    packet_loss 0.017
  ]
  edge [
    source 16
    target 30
    latency "149 ms"
    packet_loss 0.0046
  ]
  edge [
    source 16
    target 31
    latency "18 ms"
    packet_loss 0.0458
  ]
  edge [
    source 16
    target 32
    latency "84 ms"
    packet_loss 0.0411
  ]
  edge [
    source 16
    target 33
    latency "20 ms"
    packet_loss 0.0347
  ]
  edge [
    source 16
    target 34
    latency "2 ms"
    packet_loss 0.0204
  ]
  edge [
    source 16
    target 35
    latency "67 ms"
    packet_loss 0.049
  ]
  edge [
    source 16
    target 36
    latency "14 ms"
    packet_loss 0.0168
  ]
  edge [
    source 16
    target 37
    latency "183 ms"
    packet_loss 0.0189
  ]
  edge [
    source 16
    target 38
    latency "265 ms"
    packet_loss 0.0235
  ]
  edge [
    source 16
    target 39
    latency "81 ms"
    packet_loss 0.0259
  ]
  edge [
    source 16
    target 40
    latency "204 ms"
    packet_loss 0.05
  ]
  edge [
    source 16
    target 41
    latency "255 ms"
    packet_loss 0.0334
  ]
  edge [
    source 16
    target 42
    latency "98 ms"
    packet_loss 0.0186
  ]
  edge [
    source 16
    target 43
    latency "26 ms"
    packet_loss 0.0105
  ]
  edge [
    source 16
    target 44
    latency "158 ms"
    packet_loss 0.0426
  ]
  edge [
    source 16
    target 45
    latency "298 ms"
    packet_loss 0.0383
  ]
  edge [
    source 16
    target 46
    latency "150 ms"
    packet_loss 0.0129
  ]
  edge [
    source 16
    target 47
    latency "111 ms"
    packet_loss 0.0308
  ]
  edge [
    source 16
    target 48
    latency "288 ms"
    packet_loss 0.0106
  ]
  edge [
    source 16
    target 49
    latency "188 ms"
    packet_loss 0.0048
  ]
  edge [
    source 17
    target 17
    latency "6 ms"
    packet_loss 0.0352
  ]
  edge [
    source 17
    target 18
    latency "191 ms"
    packet_loss 0.0458
  ]
  edge [
    source 17
    target 19
    latency "294 ms"
    packet_loss 0.0489
  ]
  edge [
    source 17
    target 20
    latency "123 ms"
    packet_loss 0.0283
  ]
  edge [
    source 17
    target 21
    latency "149 ms"
    packet_loss 0.0212
  ]
  edge [
    source 17
    target 22
    latency "200 ms"
    packet_loss 0.0176
  ]
  edge [
    source 17
    target 23
    latency "165 ms"
    packet_loss 0.0019
  ]
  edge [
    source 17
    target 24
    latency "200 ms"
    packet_loss 0.0426
  ]
  edge [
    source 17
    target 25
    latency "175 ms"
    packet_loss 0.0494
  ]
  edge [
    source 17
    target 26
    latency "265 ms"
    packet_loss 0.0313
  ]
  edge [
    source 17
    target 27
    latency "192 ms"
    packet_loss 0.0141
  ]
  edge [
    source 17
    target 28
    latency "65 ms"
    packet_loss 0.039
  ]
  edge [
    source 17
    target 29
    latency "177 ms"
    packet_loss 0.007
  ]
  edge [
    source 17
    target 30
    latency "299 ms"
    packet_loss 0.0219
  ]
  edge [
    source 17
    target 31
    latency "104 ms"
    packet_loss 0.0402
  ]
  edge [
    source 17
    target 32
    latency "109 ms"
    packet_loss 0.0076
  ]
  edge [
    source 17
    target 33
    latency "234 ms"
    packet_loss 0.0497
  ]
  edge [
    source 17
    target 34
    latency "170 ms"
    packet_loss 0.0322
  ]
  edge [
    source 17
    target 35
    latency "138 ms"
    packet_loss 0.0082
  ]
  edge [
    source 17
    target 36
    latency "270 ms"
    packet_loss 0.0285
  ]
  edge [
    source 17
    target 37
    latency "126 ms"
    packet_loss 0.0224
  ]
  edge [
    source 17
    target 38
    latency "169 ms"
    packet_loss 0.034
  ]
  edge [
    source 17
    target 39
    latency "207 ms"
    packet_loss 0.0399
  ]
  edge [
    source 17
    target 40
    latency "34 ms"
    packet_loss 0.0349
  ]
  edge [
    source 17
    target 41
    latency "294 ms"
    packet_loss 0.0238
  ]
  edge [
    source 17
    target 42
    latency "248 ms"
    packet_loss 0.0062
  ]
  edge [
    source 17
    target 43
    latency "204 ms"
    packet_loss 0.0205
  ]
  edge [
    source 17
    target 44
    latency "256 ms"
    packet_loss 0.0109
  ]
  edge [
    source 17
    target 45
    latency "196 ms"
    packet_loss 0.0322
  ]
  edge [
    source 17
    target 46
    latency "101 ms"
    packet_loss 0.0137
  ]
  edge [
    source 17
    target 47
    latency "112 ms"
    packet_loss 0.0345
  ]
  edge [
    source 17
    target 48
    latency "5 ms"
    packet_loss 0.0198
  ]
  edge [
    source 17
    target 49
    latency "143 ms"
    packet_loss 0.0387
  ]
  edge [
    source 18
    target 18
    latency "3 ms"
    packet_loss 0.0317
  ]
  edge [
    source 18
    target 19
    latency "177 ms"
    packet_loss 0.0061
  ]
  edge [
    source 18
    target 20
    latency "17 ms"
    packet_loss 0.0126
  ]
  edge [
    source 18
    target 21
    latency "12 ms"
    packet_loss 0.0139
  ]
  edge [
    source 18
    target 22
    latency "71 ms"
    packet_loss 0.024
  ]
  edge [
    source 18
    target 23
    latency "72 ms"
    packet_loss 0.0391
  ]
  edge [
    source 18
    target 24
    latency "219 ms"
    packet_loss 0.0216
  ]
  edge [
    source 18
    target 25
    latency "246 ms"
    packet_loss 0.0409
  ]
  edge [
    source 18
    target 26
    latency "176 ms"
    packet_loss 0.0001
  ]
  edge [
    source 18
    target 27
    latency "217 ms"
    packet_loss 0.0421
  ]
  edge [
    source 18
    target 28
    latency "4 ms"
    packet_loss 0.0289
  ]
  edge [
    source 18
    target 29
    latency "242 ms"
    packet_loss 0.0129
  ]
  edge [
    source 18
    target 30
    latency "112 ms"
    packet_loss 0.0351
  ]
  edge [
    source 18
    target 31
    latency "170 ms"
    packet_loss 0.04
  ]
  edge [
    source 18
    target 32
    latency "20 ms"
    packet_loss 0.0171
  ]
  edge [
    source 18
    target 33
    latency "30 ms"
    packet_loss 0.0295
  ]
  edge [
    source 18
    target 34
    latency "250 ms"
    packet_loss 0.0054
  ]
  edge [
    source 18
    target 35
    latency "7 ms"
    packet_loss 0.0128
  ]
  edge [
    source 18
    target 36
    latency "180 ms"
    packet_loss 0.0407
  ]
  edge [
    source 18
    target 37
    latency "158 ms"
    packet_loss 0.0359
  ]
  edge [
    source 18
    target 38
    latency "31 ms"
    packet_loss 0.0141
  ]
  edge [
    source 18
    target 39
    latency "185 ms"
    packet_loss 0.0424
  ]
  edge [
    source 18
    target 40
    latency "88 ms"
    packet_loss 0.0466
  ]
  edge [
    source 18
    target 41
    latency "29 ms"
    packet_loss 0.0018
  ]
  edge [
    source 18
    target 42
    latency "258 ms"
    packet_loss 0.0175
  ]
  edge [
    source 18
    target 43
    latency "24 ms"
    packet_loss 0.0354
  ]
  edge [
    source 18
    target 44
    latency "101 ms"
    packet_loss 0.0082
  ]
  edge [
    source 18
    target 45
    latency "181 ms"
    packet_loss 0.0488
  ]
  edge [
    source 18
    target 46
    latency "219 ms"
    packet_loss 0.0177
  ]
  edge [
    source 18
    target 47
    latency "33 ms"
    packet_loss 0.0404
  ]
  edge [
    source 18
    target 48
    latency "267 ms"
    packet_loss 0.0495
  ]
  edge [
    source 18
    target 49
    latency "202 ms"
    packet_loss 0.0156
  ]
  edge [
    source 19
    target 19
    latency "7 ms"
    packet_loss 0.0464
  ]
  edge [
    source 19
    target 20
    latency "52 ms"
    packet_loss 0.0088
  ]
  edge [
    source 19
    target 21
    latency "12 ms"
    packet_loss 0.0052
  ]
  edge [
    source 19
    target 22
    latency "50 ms"
    packet_loss 0.0092
  ]
  edge [
    source 19
    target 23
    latency "132 ms"
    packet_loss 0.0417
  ]
  edge [
    source 19
    target 24
    latency "81 ms"
    packet_loss 0.0039
  ]
  edge [
    source 19
    target 25
    latency "201 ms"
    packet_loss 0.0101
  ]
  edge [
    source 19
    target 26
    latency "124 ms"
    packet_loss 0.0288
  ]
  edge [
    source 19
    target 27
    latency "191 ms"
    packet_loss 0.0358
  ]
  edge [
    source 19
    target 28
    latency "229 ms"
    packet_loss 0.025
  ]
  edge [
    source 19
    target 29
    latency "111 ms"
    packet_loss 0.0114
  ]
  edge [
    source 19
    target 30
    latency "209 ms"
    packet_loss 0.0043
  ]
  edge [
    source 19
    target 31
    latency "71 ms"
    packet_loss 0.0296
  ]
  edge [
    source 19
    target 32
    latency "24 ms"
    packet_loss 0.0178
  ]
  edge [
    source 19
    target 33
    latency "59 ms"
    packet_loss 0.0355
  ]
  edge [
    source 19
    target 34
    latency "252 ms"
    packet_loss 0.0086
  ]
  edge [
    source 19
    target 35
    latency "223 ms"
    packet_loss 0.0215
  ]
  edge [
    source 19
    target 36
    latency "181 ms"
    packet_loss 0.0248
  ]
  edge [
    source 19
    target 37
    latency "18 ms"
    packet_loss 0.0439
  ]
  edge [
    source 19
    target 38
    latency "160 ms"
    packet_loss 0.0422
  ]
  edge [
    source 19
    target 39
    latency "97 ms"
    packet_loss 0.0136
  ]
  edge [
    source 19
    target 40
    latency "170 ms"
    packet_loss 0.01
  ]
  edge [
    source 19
    target 41
    latency "69 ms"
    packet_loss 0.0249
  ]
  edge [
    source 19
    target 42
    latency "120 ms"
    packet_loss 0.0256
  ]
  edge [
    source 19
    target 43
    latency "240 ms"
    packet_loss 0.0024
  ]
  edge [
    source 19
    target 44
    latency "187 ms"
    packet_loss 0.0466
  ]
  edge [
    source 19
    target 45
    latency "197 ms"
    packet_loss 0.0362
  ]
  edge [
    source 19
    target 46
    latency "154 ms"
    packet_loss 0.0355
  ]
  edge [
    source 19
    target 47
    latency "229 ms"
    packet_loss 0.0481
  ]
  edge [
    source 19
    target 48
    latency "51 ms"
    packet_loss 0.0022
  ]
  edge [
    source 19
    target 49
    latency "22 ms"
    packet_loss 0.042
  ]
  edge [
    source 20
    target 20
    latency "10 ms"
    packet_loss 0.0246
  ]
  edge [
    source 20
    target 21
    latency "277 ms"
    packet_loss 0.0003
  ]
  edge [
    source 20
    target 22
    latency "242 ms"
    packet_loss 0.0301
  ]
  edge [
    source 20
    target 23
    latency "180 ms"
    packet_loss 0.0247
  ]
  edge [
    source 20
    target 24
    latency "235 ms"
    packet_loss 0.0073
  ]
  edge [
    source 20
    target 25
    latency "236 ms"
    packet_loss 0.0391
  ]
  edge [
    source 20
    target 26
    latency "236 ms"
    packet_loss 0.0335
  ]
  edge [
    source 20
    target 27
    latency "32 ms"
    packet_loss 0.0395
  ]
  edge [
    source 20
    target 28
    latency "19 ms"
    packet_loss 0.0475
  ]
  edge [
    source 20
    target 29
    latency "40 ms"
    packet_loss 0.0156
  ]
  edge [
    source 20
    target 30
    latency "140 ms"
    packet_loss 0.0048
  ]
  edge [
    source 20
    target 31
    latency "215 ms"
    packet_loss 0.0165
  ]
  edge [
    source 20
    target 32
    latency "170 ms"
    packet_loss 0.0343
  ]
  edge [
    source 20
    target 33
    latency "193 ms"
    packet_loss 0.0181
  ]
  edge [
    source 20
    target 34
    latency "257 ms"
    packet_loss 0.0236
  ]
  edge [
    source 20
    target 35
    latency "171 ms"
    packet_loss 0.021
  ]
  edge [
    source 20
    target 36
    latency "68 ms"
    packet_loss 0.0218
  ]
  edge [
    source 20
    target 37
    latency "94 ms"
    packet_loss 0.016
  ]
  edge [
    source 20
    target 38
    latency "138 ms"
    packet_loss 0.0226
  ]
  edge [
    source 20
    target 39
    latency "8 ms"
    packet_loss 0.0197
  ]
  edge [
    source 20
    target 40
    latency "79 ms"
    packet_loss 0.0338
  ]
  edge [
    source 20
    target 41
    latency "168 ms"
    packet_loss 0.0172
  ]
  edge [
    source 20
    target 42
    latency "49 ms"
    packet_loss 0.0347
  ]
  edge [
    source 20
    target 43
    latency "300 ms"
    packet_loss 0.0377
  ]
  edge [
    source 20
    target 44
    latency "195 ms"
    packet_loss 0.0436
  ]
  edge [
    source 20
    target 45
    latency "3 ms"
    packet_loss 0.029
  ]
  edge [
    source 20
    target 46
    latency "263 ms"
    packet_loss 0.0194
  ]
  edge [
    source 20
    target 47
    latency "56 ms"
    packet_loss 0.0069
  ]
  edge [
    source 20
    target 48
    latency "62 ms"
    packet_loss 0.0193
  ]
  edge [
    source 20
    target 49
    latency "97 ms"
    packet_loss 0.0014
  ]
  edge [
    source 21
    target 21
    latency "2 ms"
    packet_loss 0.0045
  ]
  edge [
    source 21
    target 22
    latency "76 ms"
    packet_loss 0.0435
  ]
  edge [
    source 21
    target 23
    latency "6 ms"
    packet_loss 0.018
  ]
  edge [
    source 21
    target 24
    latency "97 ms"
    packet_loss 0.0263
  ]
  edge [
    source 21
    target 25
    latency "242 ms"
    packet_loss 0.0173
  ]
  edge [
    source 21
    target 26
    latency "68 ms"
    packet_loss 0.0376
  ]
  edge [
    source 21
    target 27
    latency "175 ms"
    packet_loss 0.0381
  ]
  edge [
    source 21
    target 28
    latency "170 ms"
    packet_loss 0.044
  ]
  edge [
    source 21
    target 29
    latency "183 ms"
    packet_loss 0.0067
  ]
  edge [
    source 21
    target 30
    latency "284 ms"
    packet_loss 0.0145
  ]
  edge [
    source 21
    target 31
    latency "268 ms"
    packet_loss 0.024
  ]
  edge [
    source 21
    target 32
    latency "42 ms"
    packet_loss 0.0319
  ]
  edge [
    source 21
    target 33
    latency "92 ms"
    packet_loss 0.0279
  ]
  edge [
    source 21
    target 34
    latency "201 ms"
    packet_loss 0.0277
  ]
  edge [
    source 21
    target 35
    latency "279 ms"
    packet_loss 0.011
  ]
  edge [
    source 21
    target 36
    latency "134 ms"
    packet_loss 0.0288
  ]
  edge [
    source 21
    target 37
    latency "98 ms"
    packet_loss 0.0301
  ]
  edge [
    source 21
    target 38
    latency "89 ms"
    packet_loss 0.0395
  ]
  edge [
    source 21
    target 39
    latency "273 ms"
    packet_loss 0.0441
  ]
  edge [
    source 21
    target 40
    latency "210 ms"
    packet_loss 0.0192
  ]
  edge [
    source 21
    target 41
    latency "18 ms"
    packet_loss 0.0401
  ]
  edge [
    source 21
    target 42
    latency "52 ms"
    packet_loss 0.0418
  ]
  edge [
    source 21
    target 43
    latency "132 ms"
    packet_loss 0.0057
  ]
  edge [
    source 21
    target 44
    latency "74 ms"
    packet_loss 0.0315
  ]
  edge [
    source 21
    target 45
    latency "253 ms"
    packet_loss 0.0385
  ]
  edge [
    source 21
    target 46
    latency "54 ms"
    packet_loss 0.0462
  ]
  edge [
    source 21
    target 47
    latency "15 ms"
    packet_loss 0.0309
  ]
  edge [
    source 21
    target 48
    latency "207 ms"
    packet_loss 0.0039
  ]
  edge [
    source 21
    target 49
    latency "271 ms"
    packet_loss 0.0309
  ]
  edge [
    source 22
    target 22
    latency "7 ms"
    packet_loss 0.0399
  ]
  edge [
    source 22
    target 23
    latency "217 ms"
    packet_loss 0.0237
  ]
  edge [
    source 22
    target 24
    latency "284 ms"
    packet_loss 0.0163
  ]
  edge [
    source 22
    target 25
    latency "116 ms"
    packet_loss 0.0314
  ]
  edge [
    source 22
    target 26
    latency "148 ms"
    packet_loss 0.0192
  ]
  edge [
    source 22
    target 27
    latency "120 ms"
    packet_loss 0.0148
  ]
  edge [
    source 22
    target 28
    latency "292 ms"
    packet_loss 0.0207
  ]
  edge [
    source 22
    target 29
    latency "27 ms"
    packet_loss 0.0222
  ]
  edge [
    source 22
    target 30
    latency "132 ms"
    packet_loss 0.0455
  ]
  edge [
    source 22
    target 31
    latency "186 ms"
    packet_loss 0.0204
  ]
  edge [
    source 22
    target 32
    latency "151 ms"
    packet_loss 0.0022
  ]
  edge [
    source 22
    target 33
    latency "203 ms"
    packet_loss 0.0235
  ]
  edge [
    source 22
    target 34
    latency "221 ms"
    packet_loss 0.0407
  ]
  edge [
    source 22
    target 35
    latency "296 ms"
    packet_loss 0.0194
  ]
  edge [
    source 22
    target 36
    latency "284 ms"
    packet_loss 0.0233
  ]
  edge [
    source 22
    target 37
    latency "123 ms"
    packet_loss 0.0173
  ]
  edge [
    source 22
    target 38
    latency "286 ms"
    packet_loss 0.0481
  ]
  edge [
    source 22
    target 39
    latency "193 ms"
    packet_loss 0.0433
  ]
  edge [
    source 22
    target 40
    latency "194 ms"
    packet_loss 0.0045
  ]
  edge [
    source 22
    target 41
    latency "144 ms"
    packet_loss 0.0162
  ]
  edge [
    source 22
    target 42
    latency "109 ms"
    packet_loss 0.039
  ]
  edge [
    source 22
    target 43
    latency "1 ms"
    packet_loss 0.0366
  ]
  edge [
    source 22
    target 44
    latency "244 ms"
    packet_loss 0.0041
  ]
  edge [
    source 22
    target 45
    latency "15 ms"
    packet_loss 0.0229
  ]
  edge [
    source 22
    target 46
    latency "111 ms"
    packet_loss 0.015
  ]
  edge [
    source 22
    target 47
    latency "81 ms"
    packet_loss 0.0461
  ]
  edge [
    source 22
    target 48
    latency "219 ms"
    packet_loss 0.0088
  ]
  edge [
    source 22
    target 49
    latency "136 ms"
    packet_loss 0.0246
  ]
  edge [
    source 23
    target 23
    latency "1 ms"
    packet_loss 0.0486
  ]
  edge [
    source 23
    target 24
    latency "246 ms"
    packet_loss 0.0487
  ]
  edge [
    source 23
    target 25
    latency "178 ms"
    packet_loss 0.0115
  ]
  edge [
    source 23
    target 26
    latency "270 ms"
    packet_loss 0.038
  ]
  edge [
    source 23
    target 27
    latency "222 ms"
    packet_loss 0.0295
  ]
  edge [
    source 23
    target 28
    latency "140 ms"
    packet_loss 0.0494
  ]
  edge [
    source 23
    target 29
    latency "58 ms"
    packet_loss 0.0425
  ]
  edge [
    source 23
    target 30
    latency "36 ms"
    packet_loss 0.0015
  ]
  edge [
    source 23
    target 31
    latency "210 ms"
    packet_loss 0.0348
  ]
  edge [
    source 23
    target 32
    latency "187 ms"
    packet_loss 0.001
  ]
  edge [
    source 23
    target 33
    latency "285 ms"
    packet_loss 0.0422
  ]
  edge [
    source 23
    target 34
    latency "123 ms"
    packet_loss 0.0056
  ]
  edge [
    source 23
    target 35
    latency "298 ms"
    packet_loss 0.0162
  ]
  edge [
    source 23
    target 36
    latency "158 ms"
    packet_loss 0.014
  ]
  edge [
    source 23
    target 37
    latency "33 ms"
    packet_loss 0.0416
  ]
  edge [
    source 23
    target 38
    latency "57 ms"
    packet_loss 0.0428
  ]
  edge [
    source 23
    target 39
    latency "92 ms"
    packet_loss 0.0477
  ]
  edge [
    source 23
    target 40
    latency "266 ms"
    packet_loss 0.0317
  ]
  edge [
    source 23
    target 41
    latency "98 ms"
    packet_loss 0.0216
  ]
  edge [
    source 23
    target 42
    latency "134 ms"
    packet_loss 0.033
  ]
  edge [
    source 23
    target 43
    latency "169 ms"
    packet_loss 0.0114
  ]
  edge [
    source 23
    target 44
    latency "10 ms"
    packet_loss 0.0201
  ]
  edge [
    source 23
    target 45
    latency "294 ms"
    packet_loss 0.0191
  ]
  edge [
    source 23
    target 46
    latency "124 ms"
    packet_loss 0.0385
  ]
  edge [
    source 23
    target 47
    latency "99 ms"
    packet_loss 0.0476
  ]
  edge [
    source 23
    target 48
    latency "281 ms"
    packet_loss 0.0283
  ]
  edge [
    source 23
    target 49
    latency "185 ms"
    packet_loss 0.0014
  ]
  edge [
    source 24
    target 24
    latency "7 ms"
    packet_loss 0.0313
  ]
  edge [
    source 24
    target 25
    latency "80 ms"
    packet_loss 0.0188
  ]
  edge [
    source 24
    target 26
    latency "271 ms"
    packet_loss 0.0345
  ]
  edge [
    source 24
    target 27
    latency "143 ms"
    packet_loss 0.002
  ]
  edge [
    source 24
    target 28
    latency "17 ms"
    packet_loss 0.0049
  ]
  edge [
    source 24
    target 29
    latency "202 ms"
    packet_loss 0.0479
  ]
  edge [
    source 24
    target 30
    latency "171 ms"
    packet_loss 0.0472
  ]
  edge [
    source 24
    target 31
    latency "150 ms"
    packet_loss 0.0328
  ]
  edge [
    source 24
    target 32
    latency "107 ms"
    packet_loss 0.0295
  ]
  edge [
    source 24
    target 33
    latency "125 ms"
    packet_loss 0.0332
  ]
  edge [
    source 24
    target 34
    latency "274 ms"
    packet_loss 0.0224
  ]
  edge [
    source 24
    target 35
    latency "249 ms"
    packet_loss 0.0002
  ]
  edge [
    source 24
    target 36
    latency "134 ms"
    packet_loss 0.0335
  ]
  edge [
    source 24
    target 37
    latency "106 ms"
    packet_loss 0.0444
  ]
  edge [
    source 24
    target 38
    latency "117 ms"
    packet_loss 0.0181
  ]
  edge [
    source 24
    target 39
    latency "6 ms"
    packet_loss 0.0111
  ]
  edge [
    source 24
    target 40
    latency "49 ms"
    packet_loss 0.0423
  ]
  edge [
    source 24
    target 41
    latency "187 ms"
    packet_loss 0.018
  ]
  edge [
    source 24
    target 42
    latency "183 ms"
    packet_loss 0.0274
  ]
  edge [
    source 24
    target 43
    latency "291 ms"
    packet_loss 0.0083
  ]
  edge [
    source 24
    target 44
    latency "53 ms"
    packet_loss 0.0316
  ]
  edge [
    source 24
    target 45
    latency "181 ms"
    packet_loss 0.0301
  ]
  edge [
    source 24
    target 46
    latency "25 ms"
    packet_loss 0.0205
  ]
  edge [
    source 24
    target 47
    latency "80 ms"
    packet_loss 0.0452
  ]
  edge [
    source 24
    target 48
    latency "200 ms"
    packet_loss 0.0397
  ]
  edge [
    source 24
    target 49
    latency "112 ms"
    packet_loss 0.0186
  ]
  edge [
    source 25
    target 25
    latency "7 ms"
    packet_loss 0.0344
  ]
  edge [
    source 25
    target 26
    latency "221 ms"
    packet_loss 0.0163
  ]
  edge [
    source 25
    target 27
    latency "139 ms"
    packet_loss 0.0239
  ]
  edge [
    source 25
    target 28
    latency "28 ms"
    packet_loss 0.0111
  ]
  edge [
    source 25
    target 29
    latency "117 ms"
    packet_loss 0.025
  ]
  edge [
    source 25
    target 30
    latency "211 ms"
    packet_loss 0.0287
  ]
  edge [
    source 25
    target 31
    latency "146 ms"
    packet_loss 0.0057
  ]
  edge [
    source 25
    target 32
    latency "66 ms"
    packet_loss 0.0312
  ]
  edge [
    source 25
    target 33
    latency "191 ms"
    packet_loss 0.0004
  ]
  edge [
    source 25
    target 34
    latency "14 ms"
    packet_loss 0.001
  ]
  edge [
    source 25
    target 35
    latency "154 ms"
    packet_loss 0.0151
  ]
  edge [
    source 25
    target 36
    latency "10 ms"
    packet_loss 0.0156
  ]
  edge [
    source 25
    target 37
    latency "232 ms"
    packet_loss 0.0041
  ]
  edge [
    source 25
    target 38
    latency "223 ms"
    packet_loss 0.0085
  ]
  edge [
    source 25
    target 39
    latency "257 ms"
    packet_loss 0.0455
  ]
  edge [
    source 25
    target 40
    latency "91 ms"
    packet_loss 0.0043
  ]
  edge [
    source 25
    target 41
    latency "15 ms"
    packet_loss 0.0003
  ]
  edge [
    source 25
    target 42
    latency "42 ms"
    packet_loss 0.0359
  ]
  edge [
    source 25
    target 43
    latency "245 ms"
    packet_loss 0.0015
  ]
  edge [
    source 25
    target 44
    latency "9 ms"
    packet_loss 0.0434
  ]
  edge [
    source 25
    target 45
    latency "224 ms"
    packet_loss 0.0301
  ]
  edge [
    source 25
    target 46
    latency "279 ms"
    packet_loss 0.0068
  ]
  edge [
    source 25
    target 47
    latency "237 ms"
    packet_loss 0.0479
  ]
  edge [
    source 25
    target 48
    latency "50 ms"
    packet_loss 0.0102
  ]
  edge [
    source 25
    target 49
    latency "89 ms"
    packet_loss 0.0343
  ]
  edge [
    source 26
    target 26
    latency "4 ms"
    packet_loss 0.019
  ]
  edge [
    source 26
    target 27
    latency "15 ms"
    packet_loss 0.0185
  ]
  edge [
    source 26
    target 28
    latency "96 ms"
    packet_loss 0.0282
  ]
  edge [
    source 26
    target 29
    latency "6 ms"
    packet_loss 0.0481
  ]
  edge [
    source 26
    target 30
    latency "168 ms"
    packet_loss 0.0382
  ]
  edge [
    source 26
    target 31
    latency "69 ms"
    packet_loss 0.0089
  ]
  edge [
    source 26
    target 32
    latency "228 ms"
    packet_loss 0.0427
  ]
  edge [
    source 26
    target 33
    latency "95 ms"
    packet_loss 0.015
  ]
  edge [
    source 26
    target 34
    latency "73 ms"
    packet_loss 0.0272
  ]
  edge [
    source 26
    target 35
    latency "187 ms"
    packet_loss 0.0339
  ]
  edge [
    source 26
    target 36
    latency "114 ms"
    packet_loss 0.0415
  ]
  edge [
    source 26
    target 37
    latency "77 ms"
    packet_loss 0.0339
  ]
  edge [
    source 26
    target 38
    latency "125 ms"
    packet_loss 0.0453
  ]
  edge [
    source 26
    target 39
    latency "258 ms"
    packet_loss 0.0355
  ]
  edge [
    source 26
    target 40
    latency "256 ms"
    packet_loss 0.0172
  ]
  edge [
    source 26
    target 41
    latency "146 ms"
    packet_loss 0.0355
  ]
  edge [
    source 26
    target 42
    latency "279 ms"
    packet_loss 0.0435
  ]
  edge [
    source 26
    target 43
    latency "169 ms"
    packet_loss 0.0241
  ]
  edge [
    source 26
    target 44
    latency "28 ms"
    packet_loss 0.0231
  ]
  edge [
    source 26
    target 45
    latency "258 ms"
    packet_loss 0.0399
  ]
  edge [
    source 26
    target 46
    latency "158 ms"
    packet_loss 0.0142
  ]
  edge [
    source 26
    target 47
    latency "129 ms"
    packet_loss 0.0253
  ]
  edge [
    source 26
    target 48
    latency "106 ms"
    packet_loss 0.0471
  ]
  edge [
    source 26
    target 49
    latency "51 ms"
    packet_loss 0.0192
  ]
  edge [
    source 27
    target 27
    latency "9 ms"
    packet_loss 0.0204
  ]
  edge [
    source 27
    target 28
    latency "59 ms"
    packet_loss 0.0027
  ]
  edge [
    source 27
    target 29
    latency "78 ms"
    packet_loss 0.0118
  ]
  edge [
    source 27
    target 30
    latency "11 ms"
    packet_loss 0.0424
  ]
  edge [
    source 27
    target 31
    latency "251 ms"
    packet_loss 0.0427
  ]
  edge [
    source 27
    target 32
    latency "222 ms"
    packet_loss 0.0048
  ]
  edge [
    source 27
    target 33
    latency "38 ms"
    packet_loss 0.0388
  ]
  edge [
    source 27
    target 34
    latency "252 ms"
    packet_loss 0.0177
  ]
  edge [
    source 27
    target 35
    latency "88 ms"
    packet_loss 0.0024
  ]
  edge [
    source 27
    target 36
    latency "70 ms"
    packet_loss 0.0177
  ]
  edge [
    source 27
    target 37
    latency "130 ms"
    packet_loss 0.0075
  ]
  edge [
    source 27
    target 38
    latency "198 ms"
    packet_loss 0.0497
  ]
  edge [
    source 27
    target 39
    latency "187 ms"
    packet_loss 0.0175
  ]
  edge [
    source 27
    target 40
    latency "140 ms"
    packet_loss 0.0227
  ]
  edge [
    source 27
    target 41
    latency "108 ms"
    packet_loss 0.0401
  ]
  edge [
    source 27
    target 42
    latency "164 ms"
    packet_loss 0.0209
  ]
  edge [
    source 27
    target 43
    latency "29 ms"
    packet_loss 0.0338
  ]
  edge [
    source 27
    target 44
    latency "256 ms"
    packet_loss 0.0331
  ]
  edge [
    source 27
    target 45
    latency "247 ms"
    packet_loss 0.0015
  ]
  edge [
    source 27
    target 46
    latency "11 ms"
    packet_loss 0.0359
  ]
  edge [
    source 27
    target 47
    latency "159 ms"
    packet_loss 0.0263
  ]
  edge [
    source 27
    target 48
    latency "289 ms"
    packet_loss 0.0064
  ]
  edge [
    source 27
    target 49
    latency "169 ms"
    packet_loss 0.0423
  ]
  edge [
    source 28
    target 28
    latency "1 ms"
    packet_loss 0.0305
  ]
  edge [
    source 28
    target 29
    latency "24 ms"
    packet_loss 0.0093
  ]
  edge [
    source 28
    target 30
    latency "71 ms"
    packet_loss 0.0065
  ]
  edge [
    source 28
    target 31
    latency "36 ms"
    packet_loss 0.04
  ]
  edge [
    source 28
    target 32
    latency "250 ms"
    packet_loss 0.0071
  ]
  edge [
    source 28
    target 33
    latency "251 ms"
    packet_loss 0.0017
  ]
  edge [
    source 28
    target 34
    latency "181 ms"
    packet_loss 0.0328
  ]
  edge [
    source 28
    target 35
    latency "138 ms"
    packet_loss 0.0365
  ]
  edge [
    source 28
    target 36
    latency "146 ms"
    packet_loss 0.0207
  ]
  edge [
    source 28
    target 37
    latency "22 ms"
    packet_loss 0.0244
  ]
  edge [
    source 28
    target 38
    latency "89 ms"
    packet_loss 0.0169
  ]
  edge [
    source 28
    target 39
    latency "80 ms"
    packet_loss 0.0104
  ]
  edge [
    source 28
    target 40
    latency "33 ms"
    packet_loss 0.0021
  ]
  edge [
    source 28
    target 41
    latency "243 ms"
    packet_loss 0.026
  ]
  edge [
    source 28
    target 42
    latency "140 ms"
    packet_loss 0.0276
  ]
  edge [
    source 28
    target 43
    latency "3 ms"
    packet_loss 0.0083
  ]
  edge [
    source 28
    target 44
    latency "129 ms"
    packet_loss 0.0073
  ]
  edge [
    source 28
    target 45
    latency "141 ms"
    packet_loss 0.0257
  ]
  edge [
    source 28
    target 46
    latency "205 ms"
    packet_loss 0.0367
  ]
  edge [
    source 28
    target 47
    latency "145 ms"
    packet_loss 0.0435
  ]
  edge [
    source 28
    target 48
    latency "140 ms"
    packet_loss 0.0367
  ]
  edge [
    source 28
    target 49
    latency "256 ms"
    packet_loss 0.0489
  ]
  edge [
    source 29
    target 29
    latency "10 ms"
    packet_loss 0.0309
  ]
  edge [
    source 29
    target 30
    latency "96 ms"
    packet_loss 0.0201
  ]
  edge [
    source 29
    target 31
    latency "187 ms"
    packet_loss 0.0048
  ]
  edge [
    source 29
    target 32
    latency "144 ms"
    packet_loss 0.0433
  ]
  edge [
    source 29
    target 33
    latency "239 ms"
    packet_loss 0.046
  ]
  edge [
    source 29
    target 34
    latency "144 ms"
    packet_loss 0.0038
  ]
  edge [
    source 29
    target 35
    latency "192 ms"
    packet_loss 0.0397
  ]
  edge [
    source 29
    target 36
    latency "90 ms"
    packet_loss 0.0049
  ]
  edge [
    source 29
    target 37
    latency "282 ms"
    packet_loss 0.0135
  ]
  edge [
    source 29
    target 38
    latency "109 ms"
    packet_loss 0.0032
  ]
  edge [
    source 29
    target 39
    latency "182 ms"
    packet_loss 0.0148
  ]
  edge [
    source 29
    target 40
    latency "90 ms"
    packet_loss 0.037
  ]
  edge [
    source 29
    target 41
    latency "141 ms"
    packet_loss 0.012
  ]
  edge [
    source 29
    target 42
    latency "173 ms"
    packet_loss 0.0366
  ]
  edge [
    source 29
    target 43
    latency "66 ms"
    packet_loss 0.026
  ]
  edge [
    source 29
    target 44
    latency "24 ms"
    packet_loss 0.0154
  ]
  edge [
    source 29
    target 45
    latency "116 ms"
    packet_loss 0.0323
  ]
  edge [
    source 29
    target 46
    latency "230 ms"
    packet_loss 0.0486
  ]
  edge [
    source 29
    target 47
    latency "226 ms"
    packet_loss 0.0428
  ]
  edge [
    source 29
    target 48
    latency "227 ms"
    packet_loss 0.0208
  ]
  edge [
    source 29
    target 49
    latency "221 ms"
    packet_loss 0.0242
  ]
  edge [
    source 30
    target 30
    latency "1 ms"
    packet_loss 0.0306
  ]
  edge [
    source 30
    target 31
    latency "27 ms"
    packet_loss 0.0322
  ]
  edge [
    source 30
    target 32
    latency "266 ms"
    packet_loss 0.017
  ]
  edge [
    source 30
    target 33
    latency "140 ms"
    packet_loss 0.0064
  ]
  edge [
    source 30
    target 34
    latency "49 ms"
    packet_loss 0.0046
  ]
  edge [
    source 30
    target 35
    latency "240 ms"
    packet_loss 0.0176
  ]
  edge [
    source 30
    target 36
    latency "14 ms"
    packet_loss 0.0154
  ]
  edge [
    source 30
    target 37
    latency "290 ms"
    packet_loss 0.0169
  ]
  edge [
    source 30
    target 38
    latency "244 ms"
    packet_loss 0.0464
  ]
  edge [
    source 30
    target 39
    latency "75 ms"
    packet_loss 0.0088
  ]
  edge [
    source 30
    target 40
    latency "281 ms"
    packet_loss 0.0467
  ]
  edge [
    source 30
    target 41
    latency "169 ms"
    packet_loss 0.0132
  ]
  edge [
    source 30
    target 42
    latency "11 ms"
    packet_loss 0.0171
  ]
  edge [
    source 30
    target 43
    latency "169 ms"
    packet_loss 0.0215
  ]
  edge [
    source 30
    target 44
    latency "245 ms"
    packet_loss 0.0472
  ]
  edge [
    source 30
    target 45
    latency "275 ms"
    packet_loss 0.0486
  ]
  edge [
    source 30
    target 46
    latency "226 ms"
    packet_loss 0.0138
  ]
  edge [
    source 30
    target 47
    latency "86 ms"
    packet_loss 0.0096
  ]
  edge [
    source 30
    target 48
    latency "255 ms"
    packet_loss 0.0219
  ]
  edge [
    source 30
    target 49
    latency "201 ms"
    packet_loss 0.0296
  ]
  edge [
    source 31
    target 31
    latency "3 ms"
    packet_loss 0.0062
  ]
  edge [
    source 31
    target 32
    latency "196 ms"
    packet_loss 0.0368
  ]
  edge [
    source 31
    target 33
    latency "5 ms"
    packet_loss 0.0205
  ]
  edge [
    source 31
    target 34
    latency "182 ms"
    packet_loss 0.0401
  ]
  edge [
    source 31
    target 35
    latency "143 ms"
    packet_loss 0.0309
  ]
  edge [
    source 31
    target 36
    latency "141 ms"
    packet_loss 0.0072
  ]
  edge [
    source 31
    target 37
    latency "196 ms"
    packet_loss 0.017
  ]
  edge [
    source 31
    target 38
    latency "39 ms"
    packet_loss 0.0152
  ]
  edge [
    source 31
    target 39
    latency "100 ms"
    packet_loss 0.0313
  ]
  edge [
    source 31
    target 40
    latency "196 ms"
    packet_loss 0.0464
  ]
  edge [
    source 31
    target 41
    latency "2 ms"
    packet_loss 0.0413
  ]
  edge [
    source 31
    target 42
    latency "33 ms"
    packet_loss 0.0363
  ]
  edge [
    source 31
    target 43
    latency "174 ms"
    packet_loss 0.0413
  ]
  edge [
    source 31
    target 44
    latency "256 ms"
    packet_loss 0.0132
  ]
  edge [
    source 31
    target 45
    latency "283 ms"
    packet_loss 0.0462
  ]
  edge [
    source 31
    target 46
    latency "124 ms"
    packet_loss 0.007
  ]
  edge [
    source 31
    target 47
    latency "161 ms"
    packet_loss 0.0083
  ]
  edge [
    source 31
    target 48
    latency "136 ms"
    packet_loss 0.0144
  ]
  edge [
    source 31
    target 49
    latency "205 ms"
    packet_loss 0.0259
  ]
  edge [
    source 32
    target 32
    latency "1 ms"
    packet_loss 0.0444
  ]
  edge [
    source 32
    target 33
    latency "72 ms"
    packet_loss 0.0177
  ]
  edge [
    source 32
    target 34
    latency "286 ms"
    packet_loss 0.0431
  ]
  edge [
    source 32
    target 35
    latency "83 ms"
    packet_loss 0.0181
  ]
  edge [
    source 32
    target 36
    latency "200 ms"
    packet_loss 0.0419
  ]
  edge [
    source 32
    target 37
    latency "52 ms"
    packet_loss 0.0162
  ]
  edge [
    source 32
    target 38
    latency "195 ms"
    packet_loss 0.0469
  ]
  edge [
    source 32
    target 39
    latency "264 ms"
    packet_loss 0.0113
  ]
  edge [
    source 32
    target 40
    latency "224 ms"
    packet_loss 0.0099
  ]
  edge [
    source 32
    target 41
    latency "198 ms"
    packet_loss 0.0005
  ]
  edge [
    source 32
    target 42
    latency "93 ms"
    packet_loss 0.0158
  ]
  edge [
    source 32
    target 43
    latency "290 ms"
    packet_loss 0.0382
  ]
  edge [
    source 32
    target 44
    latency "44 ms"
    packet_loss 0.0146
  ]
  edge [
    source 32
    target 45
    latency "287 ms"
    packet_loss 0.036
  ]
  edge [
    source 32
    target 46
    latency "32 ms"
    packet_loss 0.0443
  ]
  edge [
    source 32
    target 47
    latency "99 ms"
    packet_loss 0.0206
  ]
  edge [
    source 32
    target 48
    latency "89 ms"
    packet_loss 0.0026
  ]
  edge [
    source 32
    target 49
    latency "58 ms"
    packet_loss 0.0118
  ]
  edge [
    source 33
    target 33
    latency "5 ms"
    packet_loss 0.0436
  ]
  edge [
    source 33
    target 34
    latency "55 ms"
    packet_loss 0.0134
  ]
  edge [
    source 33
    target 35
    latency "243 ms"
    packet_loss 0.0098
  ]
  edge [
    source 33
    target 36
    latency "91 ms"
    packet_loss 0.0348
  ]
  edge [
    source 33
    target 37
    latency "290 ms"
    packet_loss 0.022
  ]
  edge [
    source 33
    target 38
    latency "133 ms"
    packet_loss 0.0089
  ]
  edge [
    source 33
    target 39
    latency "82 ms"
    packet_loss 0.0111
  ]
  edge [
    source 33
    target 40
    latency "160 ms"
    packet_loss 0.0469
  ]
  edge [
    source 33
    target 41
    latency "67 ms"
    packet_loss 0.0165
  ]
  edge [
    source 33
    target 42
    latency "280 ms"
    packet_loss 0.0317
  ]
  edge [
    source 33
    target 43
    latency "171 ms"
    packet_loss 0.0321
  ]
  edge [
    source 33
    target 44
    latency "127 ms"
    packet_loss 0.0362
  ]
  edge [
    source 33
    target 45
    latency "106 ms"
    packet_loss 0.0298
  ]
  edge [
    source 33
    target 46
    latency "257 ms"
    packet_loss 0.0401
  ]
  edge [
    source 33
    target 47
    latency "25 ms"
    packet_loss 0.028
  ]
  edge [
    source 33
    target 48
    latency "159 ms"
    packet_loss 0.0107
  ]
  edge [
    source 33
    target 49
    latency "181 ms"
    packet_loss 0.0442
  ]
  edge [
    source 34
    target 34
    latency "8 ms"
    packet_loss 0.0358
  ]
  edge [
    source 34
    target 35
    latency "249 ms"
    packet_loss 0.013
  ]
  edge [
    source 34
    target 36
    latency "33 ms"
    packet_loss 0.0412
  ]
  edge [
    source 34
    target 37
    latency "272 ms"
    packet_loss 0.0353
  ]
  edge [
    source 34
    target 38
    latency "161 ms"
    packet_loss 0.0256
  ]
  edge [
    source 34
    target 39
    latency "45 ms"
    packet_loss 0.033
  ]
  edge [
    source 34
    target 40
    latency "96 ms"
    packet_loss 0.0079
  ]
  edge [
    source 34
    target 41
    latency "148 ms"
    packet_loss 0.0465
  ]
  edge [
    source 34
    target 42
    latency "5 ms"
    packet_loss 0.0226
  ]
  edge [
    source 34
    target 43
    latency "247 ms"
    packet_loss 0.0328
  ]
  edge [
    source 34
    target 44
    latency "114 ms"
    packet_loss 0.0192
  ]
  edge [
    source 34
    target 45
    latency "178 ms"
    packet_loss 0.034
  ]
  edge [
    source 34
    target 46
    latency "74 ms"
    packet_loss 0.0428
  ]
  edge [
    source 34
    target 47
    latency "99 ms"
    packet_loss 0.0123
  ]
  edge [
    source 34
    target 48
    latency "88 ms"
    packet_loss 0.0083
  ]
  edge [
    source 34
    target 49
    latency "194 ms"
    packet_loss 0.0017
  ]
  edge [
    source 35
    target 35
    latency "6 ms"
    packet_loss 0.0114
  ]
  edge [
    source 35
    target 36
    latency "26 ms"
    packet_loss 0.003
  ]
  edge [
    source 35
    target 37
    latency "96 ms"
    packet_loss 0.032
  ]
  edge [
    source 35
    target 38
    latency "8 ms"
    packet_loss 0.0169
  ]
  edge [
    source 35
    target 39
    latency "108 ms"
    packet_loss 0.0472
  ]
  edge [
    source 35
    target 40
    latency "210 ms"
    packet_loss 0.0137
  ]
  edge [
    source 35
    target 41
    latency "157 ms"
    packet_loss 0.0051
  ]
  edge [
    source 35
    target 42
    latency "71 ms"
    packet_loss 0.0212
  ]
  edge [
    source 35
    target 43
    latency "201 ms"
    packet_loss 0.0285
  ]
  edge [
    source 35
    target 44
    latency "278 ms"
    packet_loss 0.0198
  ]
  edge [
    source 35
    target 45
    latency "77 ms"
    packet_loss 0.031
  ]
  edge [
    source 35
    target 46
    latency "182 ms"
    packet_loss 0.0382
  ]
  edge [
    source 35
    target 47
    latency "290 ms"
    packet_loss 0.0148
  ]
  edge [
    source 35
    target 48
    latency "57 ms"
    packet_loss 0.0168
  ]
  edge [
    source 35
    target 49
    latency "84 ms"
    packet_loss 0.0497
  ]
  edge [
    source 36
    target 36
    latency "5 ms"
    packet_loss 0.0243
  ]
  edge [
    source 36
    target 37
    latency "210 ms"
    packet_loss 0.0308
  ]
  edge [
    source 36
    target 38
    latency "134 ms"
    packet_loss 0.0402
  ]
  edge [
    source 36
    target 39
    latency "153 ms"
    packet_loss 0.0398
  ]
  edge [
    source 36
    target 40
    latency "88 ms"
    packet_loss 0.0239
  ]
  edge [
    source 36
    target 41
    latency "90 ms"
    packet_loss 0.0001
  ]
  edge [
    source 36
    target 42
    latency "230 ms"
    packet_loss 0.0434
  ]
  edge [
    source 36
    target 43
    latency "196 ms"
    packet_loss 0.0198
  ]
  edge [
    source 36
    target 44
    latency "63 ms"
    packet_loss 0.0386
  ]
  edge [
    source 36
    target 45
    latency "27 ms"
    packet_loss 0.0088
  ]
  edge [
    source 36
    target 46
    latency "293 ms"
    packet_loss 0.0346
  ]
  edge [
    source 36
    target 47
    latency "283 ms"
    packet_loss 0.0205
  ]
  edge [
    source 36
    target 48
    latency "211 ms"
    packet_loss 0.0346
  ]
  edge [
    source 36
    target 49
    latency "104 ms"
    packet_loss 0.0328
  ]
  edge [
    source 37
    target 37
    latency "5 ms"
    packet_loss 0.0354
  ]
  edge [
    source 37
    target 38
    latency "95 ms"
    packet_loss 0.0279
  ]
  edge [
    source 37
    target 39
    latency "123 ms"
    packet_loss 0.0297
  ]
  edge [
    source 37
    target 40
    latency "84 ms"
    packet_loss 0.0415
  ]
  edge [
    source 37
    target 41
    latency "138 ms"
    packet_loss 0.0348
  ]
  edge [
    source 37
    target 42
    latency "275 ms"
    packet_loss 0.0319
  ]
  edge [
    source 37
    target 43
    latency "73 ms"
    packet_loss 0.0409
  ]
  edge [
    source 37
    target 44
    latency "94 ms"
    packet_loss 0.0127
  ]
  edge [
    source 37
    target 45
    latency "79 ms"
    packet_loss 0.0234
  ]
  edge [
    source 37
    target 46
    latency "64 ms"
    packet_loss 0.0196
  ]
  edge [
    source 37
    target 47
    latency "6 ms"
    packet_loss 0.036
  ]
  edge [
    source 37
    target 48
    latency "135 ms"
    packet_loss 0.0128
  ]
  edge [
    source 37
    target 49
    latency "157 ms"
    packet_loss 0.0456
  ]
  edge [
    source 38
    target 38
    latency "9 ms"
    packet_loss 0.0213
  ]
  edge [
    source 38
    target 39
    latency "255 ms"
    packet_loss 0.0376
  ]
  edge [
    source 38
    target 40
    latency "199 ms"
    packet_loss 0.0489
  ]
  edge [
    source 38
    target 41
    latency "11 ms"
    packet_loss 0.0049
  ]
  edge [
    source 38
    target 42
    latency "49 ms"
    packet_loss 0.0212
  ]
  edge [
    source 38
    target 43
    latency "17 ms"
    packet_loss 0.0001
  ]
  edge [
    source 38
    target 44
    latency "236 ms"
    packet_loss 0.0282
  ]
  edge [
    source 38
    target 45
    latency "206 ms"
    packet_loss 0.0015
  ]
  edge [
    source 38
    target 46
    latency "254 ms"
    packet_loss 0.0326
  ]
  edge [
    source 38
    target 47
    latency "225 ms"
    packet_loss 0.0195
  ]
  edge [
    source 38
    target 48
    latency "250 ms"
    packet_loss 0.0202
  ]
  edge [
    source 38
    target 49
    latency "121 ms"
    packet_loss 0.0435
  ]
  edge [
    source 39
    target 39
    latency "6 ms"
    packet_loss 0.0169
  ]
  edge [
    source 39
    target 40
    latency "131 ms"
    packet_loss 0.0186
  ]
  edge [
    source 39
    target 41
    latency "121 ms"
    packet_loss 0.0391
  ]
  edge [
    source 39
    target 42
    latency "223 ms"
    packet_loss 0.0016
  ]
  edge [
    source 39
    target 43
    latency "19 ms"
    packet_loss 0.0193
  ]
  edge [
    source 39
    target 44
    latency "223 ms"
    packet_loss 0.0283
  ]
  edge [
    source 39
    target 45
    latency "80 ms"
    packet_loss 0.0259
  ]
  edge [
    source 39
    target 46
    latency "26 ms"
    packet_loss 0.0106
  ]
  edge [
    source 39
    target 47
    latency "149 ms"
    packet_loss 0.0313
  ]
  edge [
    source 39
    target 48
    latency "57 ms"
    packet_loss 0.0441
  ]
  edge [
    source 39
    target 49
    latency "116 ms"
    packet_loss 0.0223
  ]
  edge [
    source 40
    target 40
    latency "8 ms"
    packet_loss 0.0121
  ]
  edge [
    source 40
    target 41
    latency "205 ms"
    packet_loss 0.0357
  ]
  edge [
    source 40
    target 42
    latency "255 ms"
    packet_loss 0.0174
  ]
  edge [
    source 40
    target 43
    latency "81 ms"
    packet_loss 0.0301
  ]
  edge [
    source 40
    target 44
    latency "281 ms"
    packet_loss 0.034
  ]
  edge [
    source 40
    target 45
    latency "47 ms"
    packet_loss 0.035
  ]
  edge [
    source 40
    target 46
    latency "210 ms"
    packet_loss 0.0427
  ]
  edge [
    source 40
    target 47
    latency "247 ms"
    packet_loss 0.0255
  ]
  edge [
    source 40
    target 48
    latency "121 ms"
    packet_loss 0.0096
  ]
  edge [
    source 40
    target 49
    latency "215 ms"
    packet_loss 0.0162
  ]
  edge [
    source 41
    target 41
    latency "7 ms"
    packet_loss 0.0364
  ]
  edge [
    source 41
    target 42
    latency "171 ms"
    packet_loss 0.0062
  ]
  edge [
    source 41
    target 43
    latency "214 ms"
    packet_loss 0.01
  ]
  edge [
    source 41
    target 44
    latency "63 ms"
    packet_loss 0.0331
  ]
  edge [
    source 41
    target 45
    latency "115 ms"
    packet_loss 0.0088
  ]
  edge [
    source 41
    target 46
    latency "19 ms"
    packet_loss 0.0352
  ]
  edge [
    source 41
    target 47
    latency "13 ms"
    packet_loss 0.0344
  ]
  edge [
    source 41
    target 48
    latency "139 ms"
    packet_loss 0.0242
  ]
  edge [
    source 41
    target 49
    latency "103 ms"
    packet_loss 0.0197
  ]
  edge [
    source 42
    target 42
    latency "7 ms"
    packet_loss 0.0347
  ]
  edge [
    source 42
    target 43
    latency "144 ms"
    packet_loss 0.0123
  ]
  edge [
    source 42
    target 44
    latency "50 ms"
    packet_loss 0.0112
  ]
  edge [
    source 42
    target 45
    latency "299 ms"
    packet_loss 0.0218
  ]
  edge [
    source 42
    target 46
    latency "75 ms"
    packet_loss 0.0154
  ]
  edge [
    source 42
    target 47
    latency "157 ms"
    packet_loss 0.0096
  ]
  edge [
    source 42
    target 48
    latency "175 ms"
    packet_loss 0.0441
  ]
  edge [
    source 42
    target 49
    latency "265 ms"
    packet_loss 0.0078
  ]
  edge [
    source 43
    target 43
    latency "4 ms"
    packet_loss 0.0283
  ]
  edge [
    source 43
    target 44
    latency "216 ms"
    packet_loss 0.0146
  ]
  edge [
    source 43
    target 45
    latency "279 ms"
    packet_loss 0.0012
  ]
  edge [
    source 43
    target 46
    latency "99 ms"
    packet_loss 0.0251
  ]
  edge [
    source 43
    target 47
    latency "264 ms"
    packet_loss 0.0316
  ]
  edge [
    source 43
    target 48
    latency "2 ms"
    packet_loss 0.0279
  ]
  edge [
    source 43
    target 49
    latency "22 ms"
    packet_loss 0.0289
  ]
  edge [
    source 44
    target 44
    latency "5 ms"
    packet_loss 0.037
  ]
  edge [
    source 44
    target 45
    latency "269 ms"
    packet_loss 0.0425
  ]
  edge [
    source 44
    target 46
    latency "91 ms"
    packet_loss 0.0103
  ]
  edge [
    source 44
    target 47
    latency "164 ms"
    packet_loss 0.0293
  ]
  edge [
    source 44
    target 48
    latency "296 ms"
    packet_loss 0.0486
  ]
  edge [
    source 44
    target 49
    latency "243 ms"
    packet_loss 0.0266
  ]
  edge [
    source 45
    target 45
    latency "8 ms"
    packet_loss 0.0499
  ]
  edge [
    source 45
    target 46
    latency "286 ms"
    packet_loss 0.0009
  ]
  edge [
    source 45
    target 47
    latency "12 ms"
    packet_loss 0.033
  ]
  edge [
    source 45
    target 48
    latency "221 ms"
    packet_loss 0.0368
  ]
  edge [
    source 45
    target 49
    latency "184 ms"
    packet_loss 0.019
  ]
  edge [
    source 46
    target 46
    latency "2 ms"
    packet_loss 0.0364
  ]
  edge [
    source 46
    target 47
    latency "83 ms"
    packet_loss 0.0018
  ]
  edge [
    source 46
    target 48
    latency "283 ms"
    packet_loss 0.0217
  ]
  edge [
    source 46
    target 49
    latency "158 ms"
    packet_loss 0.0028
  ]
  edge [
    source 47
    target 47
    latency "9 ms"
    packet_loss 0.0125
  ]
  edge [
    source 47
    target 48
    latency "281 ms"
    packet_loss 0.0178
  ]
  edge [
    source 47
    target 49
    latency "56 ms"
    packet_loss 0.0323
  ]
  edge [
    source 48
    target 48
    latency "2 ms"
    packet_loss 0.0014
  ]
  edge [
    source 48
    target 49
    latency "218 ms"
    packet_loss 0.0439
  ]
  edge [
    source 49
    target 49
    latency "7 ms"
    packet_loss 0.0371
  ]
]
